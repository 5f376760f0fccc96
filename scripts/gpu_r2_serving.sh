#!/bin/bash
# co-serving (BASELINE config 5) with chunked-prefill interleave: fp8 7B + bf16 3B behind FastAPI
export TMPDIR=/tmp
O=gpurun_out/serve; mkdir -p $O
timeout -k 10 600 python -u -m llm_based_apache_spark_optimization_amd.bench_serving --qps 4,8,16,24 --duration 20 > $O/coserve.json 2> $O/coserve.err
echo "coserve rc=$?"; tail -c 3000 $O/coserve.json

#!/bin/bash
# co-serving A/B at 16 QPS: chunked-prefill interleave and W8A8 prefill on/off
export TMPDIR=/tmp
O=gpurun_out/serveab; mkdir -p $O
run() { tag=$1; shift; env "$@" timeout -k 10 240 python -u -m llm_based_apache_spark_optimization_amd.bench_serving --qps 16 --duration 15 > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -n 5 $O/$tag.err; exit 1; }
  python -c "import json; p=json.load(open('$O/$tag.json')); print('$tag', p['achieved_qps'], p['output_tokens_per_sec'], 'nl2sql', p['nl2sql']['p50_s'], p['nl2sql']['p99_s'], 'explain', p['explain_error']['p50_s'])"; }
run nochunk LSA_PREFILL_CHUNK=0
run nochunk_w8a16 LSA_PREFILL_CHUNK=0 LSA_FP8_W8A8=0
run chunk2048 LSA_PREFILL_CHUNK=2048
run nochunk_normlaunch LSA_PREFILL_CHUNK=0 LSA_FUSED_NORM=0

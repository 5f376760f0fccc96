#!/bin/bash
# fp8 (W8A16) decode GEMM with wide n-groups: tests + sweep at the decode buckets; bench.
export TMPDIR=/tmp
O=gpurun_out/fp8wide
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fp8" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 30 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log
timeout -k 10 900 python -u scripts/bench_fp8_decode.py 1,32 > $O/sweep.jsonl 2>&1 || { tail -n 20 $O/sweep.jsonl; exit 2; }
cat $O/sweep.jsonl

#!/bin/bash
# Wide n-group skinny GEMM (nb 6 / 8: one activation fragment feeds more weight fragments) at M = 32.
export TMPDIR=/tmp
O=gpurun_out/widenb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "skinny or xfrag" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 30 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log
LSA_SWEEP_NBS=2,4,6,8 timeout -k 10 700 python -u scripts/bench_gemm_buckets.py 32 bf16 > $O/sweep_m32.jsonl 2>&1 || { tail -n 20 $O/sweep_m32.jsonl; exit 2; }
cat $O/sweep_m32.jsonl

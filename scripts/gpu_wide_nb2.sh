#!/bin/bash
# Wide n-groups for the residual epilogue (M = 32) and for batch <= 16 (nb 8, one row tile).
export TMPDIR=/tmp
O=gpurun_out/widenb2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "xfrag or rownorm or skinny" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 30 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log
timeout -k 10 600 python -u scripts/bench_res_epi.py 1,8,16,32 bf16 --rowp-only > $O/res.jsonl 2>&1 || { tail -n 20 $O/res.jsonl; exit 2; }
cat $O/res.jsonl
LSA_SWEEP_NBS=1,2,4,8 timeout -k 10 600 python -u scripts/bench_gemm_buckets.py 1,8,16 bf16 > $O/sweep_s.jsonl 2>&1 || { tail -n 20 $O/sweep_s.jsonl; exit 3; }
cat $O/sweep_s.jsonl

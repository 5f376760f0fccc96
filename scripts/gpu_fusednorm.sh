#!/bin/bash
# Norm-folded decode: kernel tests of the new epilogues, prod-shape numerics, GEMM A/B, bench.
export TMPDIR=/tmp
O=gpurun_out/fn2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "rownorm or raw_mode or skinny or silu or xfrag or fp8" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 30 $O/kern.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_prod_shapes_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/eng.log 2>&1 || { echo "engine tests failed"; tail -n 30 $O/eng.log; exit 2; }
timeout -k 10 200 python -u bench.py > $O/bench_fused.log 2>&1 || exit 4
LSA_FUSED_NORM=0 timeout -k 10 200 python -u bench.py > $O/bench_unfused.log 2>&1 || exit 5
tail -n 1 $O/bench_fused.log; tail -n 1 $O/bench_unfused.log
timeout -k 10 600 python -u scripts/bench_res_epi.py 1,8,32 bf16 > $O/res_epi_bf16.jsonl 2>&1 || exit 3

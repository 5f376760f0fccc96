#!/bin/bash
# W8A8 decode: kernel tests, engine fp8 tests, GEMM sweep, fp8 bench.
export TMPDIR=/tmp
O=gpurun_out/a8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "xf8 or fp8a or fp8_output or fp8" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 40 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_prod_shapes_gpu.py -x -q --timeout 200 --timeout-method thread > $O/eng.log 2>&1 || { echo "engine tests failed"; tail -n 40 $O/eng.log; exit 2; }
tail -n 1 $O/eng.log
timeout -k 10 600 python -u scripts/bench_fp8a_decode.py 20,32,64 > $O/sweep.jsonl 2>&1 || { tail -n 20 $O/sweep.jsonl; exit 3; }
grep shape $O/sweep.jsonl
timeout -k 10 200 python -u bench.py --dtype fp8 > $O/bench_fp8.log 2>&1 || { tail -n 20 $O/bench_fp8.log; exit 4; }
tail -n 1 $O/bench_fp8.log
LSA_FP8_A8=0 timeout -k 10 200 python -u bench.py --dtype fp8 > $O/bench_fp8_w8a16.log 2>&1 || { tail -n 20 $O/bench_fp8_w8a16.log; exit 5; }
tail -n 1 $O/bench_fp8_w8a16.log

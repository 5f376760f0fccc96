#!/bin/bash
# W8A8 decode limited to buckets > 32: production-shape decode tests incl. batch 48, engine tests, fp8 benches.
export TMPDIR=/tmp
O=gpurun_out/a8b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_prod_shapes_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/eng.log 2>&1 || { echo "engine tests failed"; tail -n 40 $O/eng.log; exit 2; }
tail -n 1 $O/eng.log
timeout -k 10 200 python -u bench.py --dtype fp8 > $O/bench_fp8.log 2>&1 || { tail -n 20 $O/bench_fp8.log; exit 4; }
tail -n 1 $O/bench_fp8.log | cut -c1-200
timeout -k 10 300 python -u bench.py --dtype fp8 --batch 64 > $O/bench_fp8_b64.log 2>&1 || { tail -n 20 $O/bench_fp8_b64.log; exit 5; }
tail -n 1 $O/bench_fp8_b64.log
LSA_FP8_A8=0 timeout -k 10 300 python -u bench.py --dtype fp8 --batch 64 > $O/bench_fp8_b64_w8a16.log 2>&1 || { tail -n 20 $O/bench_fp8_b64_w8a16.log; exit 6; }
tail -n 1 $O/bench_fp8_b64_w8a16.log

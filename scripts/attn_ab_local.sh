#!/bin/bash
# A/B of decode-attention builds (scripts/build_variants.sh): kernel tests on the default build, the
# attention microbench per variant, then the flagship bench per variant given as "$@"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attn or decode" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
for v in abvar/*.so; do
  echo "== $v"
  LSA_HIP_SO=$v timeout -k 10 120 python scripts/bench_attn.py || exit 1
done
for v in "$@"; do
  echo "== bench $v"
  LSA_HIP_SO=abvar/$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log
done

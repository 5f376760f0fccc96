#!/bin/bash
# Batch-1 attention + O projection fused: kernel test, engine / prod-shape tests, b1 A/B, profile.
export TMPDIR=/tmp
O=gpurun_out/ao
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn_o or residual or decode" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 40 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log
timeout -k 10 400 python -u -m pytest tests/test_prod_shapes_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/eng.log 2>&1 || { echo "engine tests failed"; tail -n 40 $O/eng.log; exit 2; }
tail -n 1 $O/eng.log
for v in 1 0; do
  LSA_ATTN_O=$v timeout -k 10 300 python -u bench.py --batch 1 --steps 3 --warmup 1 > $O/b1_ao$v.log 2>&1 || { tail -n 20 $O/b1_ao$v.log; exit 3; }
  echo "attn_o=$v $(tail -n1 $O/b1_ao$v.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["decode_device_ms_per_step"],d["numerics"])')"
done
bash scripts/profile_one.sh aob1 --batch 1 || exit 4

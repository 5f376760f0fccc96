#!/bin/bash
# After pack2bf = one v_cvt_pk and the exact skip-rescale: every kernel test, engine tests, attention bench, bench.
export TMPDIR=/tmp
O=gpurun_out/av3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 30 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_prod_shapes_gpu.py -x -q --timeout 200 --timeout-method thread > $O/eng.log 2>&1 || { echo "engine tests failed"; tail -n 30 $O/eng.log; exit 2; }
tail -n 1 $O/eng.log
timeout -k 10 300 python -u scripts/bench_attn_prefill.py > $O/bench_attn.jsonl 2>&1 || { tail -n 20 $O/bench_attn.jsonl; exit 3; }
grep case $O/bench_attn.jsonl
timeout -k 10 200 python -u bench.py > $O/bench.log 2>&1 || { tail -n 20 $O/bench.log; exit 4; }
tail -n 1 $O/bench.log | cut -c1-400

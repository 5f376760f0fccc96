#!/bin/bash
# Paired-group prefill attention (transposed O): kernel tests, engine prefill tests, bench paired vs single.
export TMPDIR=/tmp
O=gpurun_out/apair
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "prefill" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 30 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log


timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_prod_shapes_gpu.py -x -q --timeout 200 --timeout-method thread > $O/eng.log 2>&1 || { echo "engine tests failed"; tail -n 30 $O/eng.log; exit 3; }
tail -n 1 $O/eng.log
timeout -k 10 300 python -u scripts/bench_attn_prefill.py > $O/bench.jsonl 2>&1 || { tail -n 20 $O/bench.jsonl; exit 4; }
LSA_PREFILL_PAIR=1 timeout -k 10 300 python -u scripts/bench_attn_prefill.py > $O/bench_pair.jsonl 2>&1 || { tail -n 20 $O/bench_pair.jsonl; exit 5; }
LSA_PREFILL_PAIR=0 timeout -k 10 300 python -u scripts/bench_attn_prefill.py > $O/bench_single.jsonl 2>&1 || { tail -n 20 $O/bench_single.jsonl; exit 6; }
cat $O/bench.jsonl $O/bench_pair.jsonl $O/bench_single.jsonl | grep case

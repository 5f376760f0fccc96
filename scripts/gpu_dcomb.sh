#!/bin/bash
# Decode attention with the parallel split combine: tests, attention bench, latency benches.
export TMPDIR=/tmp
O=gpurun_out/dcomb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode or attn" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo "kernel tests failed"; tail -n 40 $O/kern.log; exit 1; }
tail -n 1 $O/kern.log
timeout -k 10 300 python -u scripts/bench_attn.py > $O/attn.jsonl 2>&1 || { tail -n 20 $O/attn.jsonl; exit 2; }
cat $O/attn.jsonl
timeout -k 10 300 python -u bench.py --model llama3.2 --batch 1 --prompt-len 2048 --steps 3 --warmup 1 > $O/explain.log 2>&1 || { tail -n 20 $O/explain.log; exit 3; }
tail -n 1 $O/explain.log | cut -c1-300
timeout -k 10 300 python -u bench.py --batch 1 --steps 3 --warmup 1 > $O/b1.log 2>&1 || { tail -n 20 $O/b1.log; exit 4; }
tail -n 1 $O/b1.log | cut -c1-300

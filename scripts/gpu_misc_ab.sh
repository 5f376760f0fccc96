#!/bin/bash
# A/Bs: short-prompt prefill attention kernel (16 vs 32 rows), norm-free vs norm launches at batch 1.
export TMPDIR=/tmp
O=gpurun_out/misc
mkdir -p $O
LSA_ATTN_CASES=7b_b32_128,3b_b4_1k LSA_PREFILL_ATTN=16 timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/p16.jsonl 2>&1 || exit 1
LSA_ATTN_CASES=7b_b32_128,3b_b4_1k LSA_PREFILL_ATTN=32 timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/p32.jsonl 2>&1 || exit 2
grep case $O/p16.jsonl $O/p32.jsonl
for fn in 1 0; do
  LSA_FUSED_NORM=$fn timeout -k 10 300 python -u bench.py --model llama3.2 --batch 1 --prompt-len 2048 --steps 3 --warmup 1 > $O/x_fn$fn.log 2>&1 || exit 3
  LSA_FUSED_NORM=$fn timeout -k 10 300 python -u bench.py --batch 1 --steps 3 --warmup 1 > $O/b1_fn$fn.log 2>&1 || exit 4
  echo "fused=$fn explain $(tail -n1 $O/x_fn$fn.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["decode_device_ms_per_step"])') b1 $(tail -n1 $O/b1_fn$fn.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["decode_device_ms_per_step"])')"
done

#!/bin/bash
# Prefill attention cost breakdown: the same bench with parts of the tile loop removed (LSA_ATTN_XMODE).
export TMPDIR=/tmp
O=gpurun_out/axm
mkdir -p $O
export LSA_ATTN_CASES=3b_explain_2k,7b_b1_2k,3b_8k
for m in 0 1 2 3 4; do
  LSA_ATTN_XMODE=$m timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/x$m.jsonl 2>&1 || { tail -n 20 $O/x$m.jsonl; exit 1; }
  echo "xmode $m"; grep case $O/x$m.jsonl
done

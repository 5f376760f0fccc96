#!/bin/bash
# Bench A/B after the wide n-group picks: 7B / 3B batch 32, norm launches vs norm-free at b32; profiles.
export TMPDIR=/tmp
O=gpurun_out/nbab
mkdir -p $O
for m in duckdb-nsql llama3.2; do
  timeout -k 10 200 python -u bench.py --model $m > $O/b32_$m.log 2>&1 || { tail -n 20 $O/b32_$m.log; exit 1; }
  LSA_FUSED_NORM_MAX_B=32 timeout -k 10 200 python -u bench.py --model $m > $O/b32_fused_$m.log 2>&1 || { tail -n 20 $O/b32_fused_$m.log; exit 2; }
  echo "$m unfused: $(tail -n 1 $O/b32_$m.log | cut -c1-200)"
  echo "$m fused:   $(tail -n 1 $O/b32_fused_$m.log | cut -c1-200)"
done
bash scripts/profile_one.sh n32 --model duckdb-nsql || exit 3
LSA_FUSED_NORM_MAX_B=32 bash scripts/profile_one.sh f32 --model duckdb-nsql || exit 4

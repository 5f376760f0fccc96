#!/bin/bash
# A/B of the decode-attention Infinity-Cache warm-up (ModelRunner.attn_prefetch_wgs) on the batch-1 configs,
# interleaved on one box: 3B 2k explain and 7B batch 1.  Output: gpurun_out/ab_attn_prefetch.txt
export TMPDIR=/tmp
out=gpurun_out/ab_attn_prefetch.txt
: > $out
for rep in 1 2; do
  for n in 0 256 512; do
    timeout -k 10 300 python -u bench.py --model llama3.2 --batch 1 --prompt-len 2048 --new-tokens 128 --steps 3 \
      --warmup 1 --no-extras --set attn_prefetch_wgs=$n > gpurun_out/ab_e_$n.log 2>&1 || { tail -20 gpurun_out/ab_e_$n.log; exit 1; }
    echo "explain wgs=$n $(tail -1 gpurun_out/ab_e_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["decode_device_ms_per_step"], d["numerics"]["ok"])')" | tee -a $out
    timeout -k 10 300 python -u bench.py --batch 1 --steps 3 --warmup 1 --no-extras --set attn_prefetch_wgs=$n \
      > gpurun_out/ab_b1_$n.log 2>&1 || { tail -20 gpurun_out/ab_b1_$n.log; exit 1; }
    echo "7b_b1 wgs=$n $(tail -1 gpurun_out/ab_b1_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["decode_device_ms_per_step"], d["numerics"]["ok"])')" | tee -a $out
  done
done

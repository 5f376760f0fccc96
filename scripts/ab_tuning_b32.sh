#!/bin/bash
# In-pipeline A/B of 7B b32 decode-GEMM configs (ops.TUNING_OVERRIDES), interleaved: the o projection
# (4096x4096 f32, fragment-major input) and the down projection (4096x11008) at 32 rows.
export TMPDIR=/tmp
out=gpurun_out/ab_tuning_b32.txt
: > $out
declare -a CFG=(
  'base={}'
  'o_4_4_8_2={"4096x4096:f32:b32:xf": {"nb": 4, "splitk": 4, "waves": 8, "div": 2}}'
  'o_2_4_4_2={"4096x4096:f32:b32:xf": {"nb": 2, "splitk": 4, "waves": 4, "div": 2}}'
  'd_2_4_8_2={"4096x11008:f32:b32:xf": {"nb": 2, "splitk": 4, "waves": 8, "div": 2}}'
)
for rep in 1 2; do
  for c in "${CFG[@]}"; do
    name=${c%%=*}; val=${c#*=}
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extras --set "ops.TUNING_OVERRIDES=$val" \
      > gpurun_out/ab_tun_$name.log 2>&1 || { tail -20 gpurun_out/ab_tun_$name.log; exit 1; }
    echo "rep=$rep $name $(tail -1 gpurun_out/ab_tun_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_device_ms_per_step"], d["numerics"]["ok"])')" | tee -a $out
  done
done

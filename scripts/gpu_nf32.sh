#!/bin/bash
# Norm-free decode at batch 32 (LSA_FUSED_NORM_MAX_B=32) vs the norm launches, 7B bf16 / 7B fp8, at HEAD.
export TMPDIR=/tmp
O=gpurun_out/nf32; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 "$@" > $O/$tag.log 2>&1 || { tail -n 20 $O/$tag.log; exit 2; }
  python - $O/$tag.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d.get("decode_device_ms_per_step"), d["numerics"]["ok"])
PY
}
for rep in 1 2; do
  run base_bf16_$rep
  LSA_FUSED_NORM_MAX_B=32 run nf_bf16_$rep
done
run base_fp8 --dtype fp8
LSA_FUSED_NORM_MAX_B=32 run nf_fp8 --dtype fp8
# decode steps per captured graph (fewer graph boundaries per token)
LSA_STEPS_PER_GRAPH=4 run spg4_bf16
LSA_STEPS_PER_GRAPH=16 run spg16_bf16

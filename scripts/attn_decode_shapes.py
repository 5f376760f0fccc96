"""Decode attention (fused RoPE + append, the engine's split plan) on the BASELINE decode shapes, us per call:
3B explain (B=1, 24/8 heads, 2k prompt + generated tokens, plan for the 2240-token window), 7B batch 1 and 32.
    python scripts/attn_decode_shapes.py > gpurun_out/attn_shapes.jsonl
"""
import json
import sys

sys.path.insert(0, "scripts")
import attn_scaling as a  # noqa: E402

for B, H, Hkv, ctx, pc in ((1, 24, 8, 2100, 2240), (1, 24, 8, 2176, 2240), (1, 32, 32, 200, 320), (32, 32, 32, 192, 320)):
    print(json.dumps({"shape": "decode", **a.run(B, H, Hkv, ctx, plan_ctx=pc)}), flush=True)

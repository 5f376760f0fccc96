"""Decode attention with the fused RoPE + KV append, bf16 cache vs fp8 cache (ops.KV_FP8), at the engine's plan
(ops.decode_split_plan of the context tier) for the BASELINE decode shapes: us per call, one JSON line per case.
The cache is spread like the serving engine's (8x the live blocks) so K/V come from HBM."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.ops import reference as ref  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, it=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    reps = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        reps.append(e0.elapsed_time(e1) * 1000 / it)
    return sorted(reps)[1]


cases = {"7b_b32_ctx200": (32, 32, 32, 200, 2), "7b_b32_ctx512": (32, 32, 32, 512, 2),
         "7b_b64_ctx200": (64, 32, 32, 200, 2), "7b_b1_ctx200": (1, 32, 32, 200, 4),
         "3b_b1_ctx2100": (1, 24, 8, 2100, 8), "3b_b32_ctx200": (32, 24, 8, 200, 8),
         "3b_b32_ctx2048": (32, 24, 8, 2048, 8)}
cos, sin = ref.rope_tables(128, 64 * max((c[3] + 63) // 64 for c in cases.values()), 500000.0, device=dev)
for name, (B, H, Hkv, ctx, nparts) in cases.items():
    nblk = (ctx + 63) // 64
    total = B * nblk * 8 + 1
    perm = torch.randperm(total - 1, device=dev)[: B * nblk].int() + 1
    bt = perm.view(B, nblk)
    pos = torch.full((B,), ctx - 1, device=dev, dtype=torch.int32)
    parts = torch.randn(nparts, B, (H + 2 * Hkv) * 128, device=dev)
    q = torch.empty(B, H, 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(q)
    tier = 256
    while tier < ctx:
        tier *= 2
    plan = ops.decode_split_plan(B, Hkv, tier)
    ws = ops.decode_workspace(B, H, Hkv, max(4, plan[1]), dev)
    kc = torch.randn(total, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    k8 = torch.randint(0, 120, (total, Hkv, 64, 128), device=dev, dtype=torch.uint8)
    v8 = torch.randint(0, 120, (total, Hkv, 64, 128), device=dev, dtype=torch.uint8)
    ks = torch.rand(total, Hkv, 64, device=dev)
    vs = torch.rand_like(ks)
    res = {"case": name, "plan": list(plan)}
    res["bf16_us"] = round(timeit(lambda: ops.attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.088, out, workspace=ws, plan=plan,
                                                          qkv_parts=parts, cos=cos, sin=sin)), 2)
    res["fp8_us"] = round(timeit(lambda: ops.attn_decode(q, k8, v8, bt, pos, H, Hkv, 0.088, out, workspace=ws, plan=plan,
                                                         qkv_parts=parts, cos=cos, sin=sin, kv_scales=(ks, vs))), 2)
    kv_bytes = B * ctx * Hkv * 128 * 2
    res["bf16_TBps"] = round(2 * kv_bytes / res["bf16_us"] / 1e6, 2)
    res["fp8_TBps"] = round((kv_bytes + B * ctx * Hkv * 8) / res["fp8_us"] / 1e6, 2)
    print(json.dumps(res), flush=True)

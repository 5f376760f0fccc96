"""Decode attention (fused RoPE + KV append from QKV slabs) vs split plan on MI355X: us per call
for the BASELINE decode shapes.  The cache is sized like the serving engine's (other sequences'
blocks in between), so K/V reads come from HBM."""
import json
import math
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


cases = {"7b_b1_ctx200": (1, 32, 32, 200, 4), "7b_b1_ctx130": (1, 32, 32, 130, 4),
         "7b_b32_ctx200": (32, 32, 32, 200, 2), "3b_b1_ctx200": (1, 24, 8, 200, 1),
         "3b_b1_ctx2100": (1, 24, 8, 2100, 8), "3b_b32_ctx200": (32, 24, 8, 200, 8)}
if len(sys.argv) > 1 and sys.argv[1] == "long":  # larger grids at longer contexts: unsplit vs split plans
    cases = {f"{m}_b{B}_ctx{c}": (B, H, Hkv, c, 2) for m, H, Hkv in (("7b", 32, 32), ("3b", 24, 8))
             for B in (8, 32) for c in (320, 512, 1024, 2048)}
    cases.update({"7b_b1_ctx1024": (1, 32, 32, 1024, 4), "7b_b1_ctx2048": (1, 32, 32, 2048, 4),
                  "7b_b4_ctx1024": (4, 32, 32, 1024, 4), "3b_b1_ctx2100": (1, 24, 8, 2100, 8),
                  "3b_b16_ctx1024": (16, 24, 8, 1024, 4), "3b_b2_ctx2048": (2, 24, 8, 2048, 8),
                  "3b_b1_ctx8192": (1, 24, 8, 8192, 8), "7b_b1_ctx200": (1, 32, 32, 200, 4)})
if len(sys.argv) > 1 and sys.argv[1] == "grid":  # 7B (G = 1) around the single-buffer grid threshold
    cases = {f"7b_b{B}_ctx{c}": (B, 32, 32, c, 2) for B in (8, 16, 24, 32, 64) for c in (200, 512)}
cos, sin = ref.rope_tables(128, 64 * max((c[3] + 63) // 64 for c in cases.values()), 500000.0, device=dev)
for name, (B, H, Hkv, ctx, nparts) in cases.items():
    nblk = (ctx + 63) // 64
    total = B * nblk * 8 + 1  # spread: 8x the live blocks
    kc = torch.randn(total, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    perm = torch.randperm(total - 1, device=dev)[: B * nblk].int() + 1
    bt = perm.view(B, nblk)
    pos = torch.full((B,), ctx - 1, device=dev, dtype=torch.int32)
    parts = torch.randn(nparts, B, (H + 2 * Hkv) * 128, device=dev)
    q = torch.empty(B, H, 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(q)
    ws = ops.decode_workspace(B, H, Hkv, 256, dev)
    res = {"case": name}
    for chunk in sorted({1, 2, 4, 8, 16, nblk}):
        if chunk > nblk or (len(sys.argv) > 1 and chunk < 2):
            continue
        nsplit = (nblk + chunk - 1) // chunk
        # unsplit threshold 0: the split is forced even for contexts of <= 4 blocks
        res[f"chunk{chunk}/split{nsplit}"] = round(timeit(lambda: ops.attn_decode(
            q, kc, vc, bt, pos, H, Hkv, 1 / math.sqrt(128), out, workspace=ws, plan=(chunk, nsplit, 0 if chunk < nblk else nblk),
            qkv_parts=parts, cos=cos, sin=sin)), 2)
    plan = ops.decode_split_plan(B, Hkv, ctx)
    res["default_plan"] = plan
    res["default_us"] = round(timeit(lambda: ops.attn_decode(
        q, kc, vc, bt, pos, H, Hkv, 1 / math.sqrt(128), out, workspace=ws, plan=plan,
        qkv_parts=parts, cos=cos, sin=sin)), 2)
    print(json.dumps(res), flush=True)

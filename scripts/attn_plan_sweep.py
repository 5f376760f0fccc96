"""Decode-attention split plans swept on the batch-1 shapes (fused RoPE + append path): us per call for forced
(chunk_blocks, nsplit, unsplit_max) plans next to ops.decode_split_plan's pick.  Re-run after a kernel change that
moves the score-loop / combine balance (e.g. the cross-lane reductions moving from ds_bpermute to DPP).
    python scripts/attn_plan_sweep.py > gpurun_out/attn_plan_sweep.jsonl
"""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from attn_scaling import cos, dev, sin, timeit  # noqa: E402


def case(name, B, H, Hkv, ctx, plan_ctx, plans):
    nblk = (ctx + 63) // 64
    total = B * nblk * 4 + 1
    kc = torch.randn(total, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = (torch.randperm(total - 1, device=dev)[: B * nblk].int() + 1).view(B, nblk)
    pos = torch.full((B,), ctx - 1, device=dev, dtype=torch.int32)
    parts = torch.randn(2, B, (H + 2 * Hkv) * 128, device=dev)
    q = torch.empty(B, H, 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(q)
    ws = ops.decode_workspace(B, H, Hkv, 256, dev)
    pick = ops.decode_split_plan(B, Hkv, plan_ctx)
    res = {"case": name, "pick": list(pick)}
    ref = None
    for _ in range(2):  # two interleaved rounds
        for p in [pick] + [pl for pl in plans if tuple(pl) != tuple(pick)]:
            kc2 = kc.clone()  # the fused append writes the new token's row: start every plan from the same cache
            vc2 = vc.clone()
            fn = lambda: ops.attn_decode(q, kc2, vc2, bt, pos, H, Hkv, 1 / math.sqrt(128), out, workspace=ws,  # noqa: E731
                                         plan=tuple(p), qkv_parts=parts, cos=cos, sin=sin)
            us = timeit(fn)
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = (out.float() - ref).abs().max().item()
            key = "x".join(str(v) for v in p)
            res.setdefault(key, []).append(round(us, 2))
            res[key + "_err"] = err
    print(json.dumps(res), flush=True)


case("3b_b1_ctx2100", 1, 24, 8, 2100, 2240, [(1, 35, 0), (2, 18, 4), (3, 12, 4), (4, 9, 4), (5, 7, 4), (6, 6, 4)])
case("7b_b1_ctx200", 1, 32, 32, 200, 320, [(1, 4, 0), (2, 2, 4), (4, 1, 4)])
case("7b_b1_ctx2100", 1, 32, 32, 2100, 2240, [(1, 35, 0), (2, 8, 4), (3, 8, 4), (4, 8, 4), (5, 7, 4), (9, 4, 4)])

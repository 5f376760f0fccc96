"""Where a decode-attention workgroup spends its time: s_memrealtime stamps (100 MHz) at 7 points of each
workgroup's critical path (csrc/kernels/attention.hip LSA_STAMP), one launch per case after warm-up.
Prints per case the median / max over workgroups of each phase (us) and the spread of start times.

    python scripts/attn_stamps.py
"""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.ops import reference as ref  # noqa: E402

dev = torch.device("cuda:0")
PH = ["start->ctx", "ctx->rope", "rope->scored", "scored->merged", "merged->ticket", "ticket->combined"]
cases = {"3b_b1_ctx2100": (1, 24, 8, 2100, 8), "7b_b1_ctx200": (1, 32, 32, 200, 4),
         "7b_b32_ctx200": (32, 32, 32, 200, 2), "3b_b32_ctx200": (32, 24, 8, 200, 8)}
cos, sin = ref.rope_tables(128, 64 * 40, 500000.0, device=dev)
for name, (B, H, Hkv, ctx, nparts) in cases.items():
    nblk = (ctx + 63) // 64
    total = B * nblk * 8 + 1
    kc = torch.randn(total, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = (torch.randperm(total - 1, device=dev)[: B * nblk].int() + 1).view(B, nblk)
    pos = torch.full((B,), ctx - 1, device=dev, dtype=torch.int32)
    parts = torch.randn(nparts, B, (H + 2 * Hkv) * 128, device=dev)
    q = torch.empty(B, H, 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(q)
    plan = ops.decode_split_plan(B, Hkv, max(256, ctx))
    ws = ops.decode_workspace(B, H, Hkv, max(plan[1], 4), dev)

    def run():
        ops.attn_decode(q, kc, vc, bt, pos, H, Hkv, 1 / math.sqrt(128), out, workspace=ws, plan=plan,
                        qkv_parts=parts, cos=cos, sin=sin)

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    st = torch.zeros(Hkv * B * plan[1] * 8, dtype=torch.int64, device=dev)
    ops.ext().attn_set_stamps(st)
    run()
    torch.cuda.synchronize()
    ops.ext().attn_set_stamps(None)
    s = st.view(-1, 8).cpu().double()
    live = s[:, 0] > 0
    s = s[live]
    t0 = s[:, 0].min()
    res = {"case": name, "plan": list(plan), "workgroups": int(live.sum()),
           "start_spread_us": round(float((s[:, 0].max() - t0) / 100), 2),
           "last_end_us": round(float((s.max(1).values.max() - t0) / 100), 2)}
    for k, ph in enumerate(PH):
        a, b = s[:, k], s[:, k + 1]
        ok = (a > 0) & (b > 0)
        if ok.any():
            d = (b[ok] - a[ok]) / 100.0
            res[ph] = [round(float(d.median()), 2), round(float(d.max()), 2), int(ok.sum())]
    print(json.dumps(res), flush=True)

# --ao: the fused batch-1 attention + O projection kernel (csrc/kernels/attention_o.hip)
if "--ao" in sys.argv:
    H, D, d, ctx = 32, 128, 4096, 200
    nblk = (ctx + 63) // 64
    kc = torch.randn(nblk * 8 + 1, H, 64, D, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = (torch.randperm(nblk * 8, device=dev)[:nblk].int() + 1).view(1, nblk)
    pos = torch.tensor([ctx - 1], dtype=torch.int32, device=dev)
    parts = torch.randn(2, 1, 3 * H * D, device=dev)
    wo = ops.PackedWeight.from_dense((torch.randn(d, H * D, device=dev) * 0.02).to(torch.bfloat16))
    h = torch.zeros(1, d, device=dev)
    x = torch.zeros(1, d, device=dev, dtype=torch.bfloat16)
    ss = torch.zeros(1, device=dev, dtype=torch.int64)
    slabs = torch.empty(H * d, device=dev)
    tk = torch.zeros(64, device=dev, dtype=torch.int32)
    for _ in range(5):
        ops.attn_o_b1(parts, cos, sin, pos, kc, vc, bt, H, 1 / math.sqrt(D), wo, slabs, tk, h, x, ss)
    torch.cuda.synchronize()
    st = torch.zeros(H * (d // 512) * 8, dtype=torch.int64, device=dev)
    ops.ext().attn_o_set_stamps(st)
    ops.attn_o_b1(parts, cos, sin, pos, kc, vc, bt, H, 1 / math.sqrt(D), wo, slabs, tk, h, x, ss)
    torch.cuda.synchronize()
    ops.ext().attn_o_set_stamps(None)
    s = st.view(-1, 8).cpu().double()
    t0 = s[:, 0].min()
    names = ["start->rope", "rope->scored", "scored->merged", "merged->ticket", "ticket->end"]
    res = {"case": "attn_o_b1_7b_ctx200", "start_spread_us": round(float((s[:, 0].max() - t0) / 100), 2),
           "last_end_us": round(float((s.max(1).values.max() - t0) / 100), 2)}
    for k, ph in enumerate(names):
        a, b = s[:, k], s[:, k + 1]
        ok = (a > 0) & (b > 0)
        if ok.any():
            dd = (b[ok] - a[ok]) / 100.0
            res[ph] = [round(float(dd.median()), 2), round(float(dd.max()), 2), int(ok.sum())]
    print(json.dumps(res), flush=True)

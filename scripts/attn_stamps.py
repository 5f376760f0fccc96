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

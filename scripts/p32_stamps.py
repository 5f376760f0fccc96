"""Per-segment cycle breakdown of the 32-row prefill attention tile loop (attention_prefill32.hip STAMP build):
for every wave, s_memtime cycles summed per segment over its tiles; reported for the heaviest groups (the causal
critical path) and averaged over all waves, per tile.  Also the stamped vs plain kernel time (the stamps' own cost).  Results and the restructurings A/B'd with it
(software-pipelined loop, one-wave-per-SIMD 512-register build, XCD-aware head placement: none faster, removed):
profiles/r5/attn_prefill_stamps_ab_mi355x.jsonl.

    python scripts/p32_stamps.py > gpurun_out/p32_stamps.jsonl
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SEG = ["dma_issue", "qk_max", "softmax", "pv_issue", "dma_wait", "barrier"]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / it


def case(name, nseq, qlen, H, Hkv):
    nblk = (qlen + 63) // 64
    total = nseq * nblk + 1
    kc = torch.randn(total, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = (torch.randperm(total - 1, device=dev)[: nseq * nblk].int() + 1).view(nseq, nblk)
    cu = [i * qlen for i in range(nseq + 1)]
    q = torch.randn(cu[-1], H, 128, device=dev).to(torch.bfloat16)
    out = torch.empty_like(q)
    cud = torch.tensor(cu, dtype=torch.int32, device=dev)
    ctx = torch.full((nseq,), qlen, dtype=torch.int32, device=dev)
    # arms: heavy / light pairing of the query blocks (ops.PREFILL_PAIR)
    ARMS = {"paired": "auto", "single": "0"}
    plans = {}
    for k, pr in ARMS.items():
        ops.PREFILL_PAIR = pr
        plans[k] = ops.prefill_plan(cu, heads=H, device=dev)
    ops.PREFILL_PAIR = "auto"

    def arm(k):
        return lambda: ops.attn_prefill(q, kc, vc, bt, cud, ctx, H, Hkv, 1 / math.sqrt(128), out, work=plans[k])

    arms = {}
    for _ in range(3):
        for k in ARMS:
            arms.setdefault(k, []).append(timeit(arm(k)))
    outs = {}
    for k in ARMS:
        out.zero_()
        arm(k)()
        torch.cuda.synchronize()
        outs[k] = out.float().clone()
    diff = {k: (outs["paired"] - outs[k]).abs().max().item() for k in ARMS}
    sel = os.environ.get("LSA_P32_STAMP_ARM", "paired")
    run = arm(sel)
    plan = plans[sel]
    ng = plan.work.shape[1] // 4
    nwork = plan.work.shape[0]
    plain = timeit(run)
    st = torch.zeros(nwork * H * ng * 4 * 8, dtype=torch.int64, device=dev)
    ops.ext().attn_prefill_set_stamps(st)
    stamped = timeit(run, it=5)
    st.zero_()
    run()
    torch.cuda.synchronize()
    ops.ext().attn_prefill_set_stamps(None)
    s = st.view(-1, 8).cpu()
    tiles = (s[:, 6] & 0xFFFFFFFF).float()
    ntmax = (s[:, 6] >> 32).float()
    rows = s[:, :6].float()
    res = {"case": name, "kernel": plan.kernel, "ng": ng, "nwork": nwork, "stamped_arm": sel, "max_diff_vs_paired": diff,
           "arms_us": {k: round(sorted(v)[1], 1) for k, v in arms.items()}, "plain_us": round(plain, 1),
           "stamped_us": round(stamped, 1)}
    # heaviest waves: the most tiles processed
    tmax = tiles.max()
    heavy = tiles == tmax
    res["heavy"] = {"waves": int(heavy.sum()), "tiles": int(tmax), "loop_iters": int(ntmax[heavy].max()),
                    "cyc_per_tile": {k: round(float(rows[heavy, i].mean() / tmax), 1) for i, k in enumerate(SEG)},
                    "kernel_cyc": round(float(s[heavy, 7].float().mean()), 0)}
    act = tiles > 0
    res["all"] = {"waves": int(act.sum()), "tiles_mean": round(float(tiles[act].mean()), 2),
                  "cyc_per_tile": {k: round(float((rows[act, i] / tiles[act]).mean()), 1) for i, k in enumerate(SEG)},
                  "kernel_cyc_mean": round(float(s[act, 7].float().mean()), 0)}
    print(json.dumps(res), flush=True)


case("3b_explain_2k", 1, 2048, 24, 8)
case("7b_b1_2k", 1, 2048, 32, 32)
if os.environ.get("LSA_P32_ALL"):
    case("3b_8k", 1, 8192, 24, 8)
    case("3b_b4_1k", 4, 1024, 24, 8)

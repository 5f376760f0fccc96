"""Prefill (causal flash) attention on MI355X: us and TFLOP/s per call for the BASELINE prefill shapes
(packed variable-length sequences over the paged cache).  Arms (interleaved per case): heavy / light query-block
pairing of the 32-row kernel (ops.PREFILL_PAIR; LSA_ATTN_PAIR=auto,0 by default)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, it=20):
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


def case(name, nseq, qlen, H, Hkv):
    if os.environ.get("LSA_ATTN_CASES") and name not in os.environ["LSA_ATTN_CASES"].split(","):
        return
    nblk = (qlen + 63) // 64
    total = nseq * nblk + 1
    kc = torch.randn(total, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = (torch.randperm(total - 1, device=dev)[: nseq * nblk].int() + 1).view(nseq, nblk)
    cu = [i * qlen for i in range(nseq + 1)]
    T = cu[-1]
    q = torch.randn(T, H, 128, device=dev).to(torch.bfloat16)
    out = torch.empty_like(q)
    cud = torch.tensor(cu, dtype=torch.int32, device=dev)
    ctx = torch.full((nseq,), qlen, dtype=torch.int32, device=dev)
    flops = nseq * 4 * H * 128 * qlen * (qlen + 1) / 2  # causal QK^T + PV
    s0 = q[:qlen].float().transpose(0, 1)
    kk = kc[bt[0].long()].transpose(0, 1).reshape(Hkv, -1, 128)[:, :qlen].float().repeat_interleave(H // Hkv, 0)
    vv = vc[bt[0].long()].transpose(0, 1).reshape(Hkv, -1, 128)[:, :qlen].float().repeat_interleave(H // Hkv, 0)
    ref = torch.nn.functional.scaled_dot_product_attention(s0, kk, vv, is_causal=True).transpose(0, 1)
    splits = os.environ.get("LSA_ATTN_PAIR", "auto,0").split(",")  # heavy / light pairing arms (ops.PREFILL_PAIR)
    plans = {}
    for sp in splits:
        ops.PREFILL_PAIR = sp
        plans[sp] = ops.prefill_plan(cu, heads=H, device=dev)
    res = {"case": name, "kernel": plans[splits[0]].kernel}
    times = {sp: [] for sp in splits}
    for _ in range(3):  # interleaved rounds
        for sp in splits:
            times[sp].append(timeit(lambda: ops.attn_prefill(q, kc, vc, bt, cud, ctx, H, Hkv, 1 / math.sqrt(128), out,
                                                              work=plans[sp])))
    for sp in splits:
        out.zero_()
        ops.attn_prefill(q, kc, vc, bt, cud, ctx, H, Hkv, 1 / math.sqrt(128), out, work=plans[sp])
        torch.cuda.synchronize()
        err = (out[:qlen].float() - ref).abs().max().item()  # spot check vs SDPA on the first sequence
        us = sorted(times[sp])[1]
        res[f"pair_{sp}"] = {"us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1), "max_err": round(err, 4),
                             "work": list(plans[sp].work.shape)}
    print(json.dumps(res), flush=True)

case("3b_explain_2k", 1, 2048, 24, 8)
case("7b_b1_2k", 1, 2048, 32, 32)
case("7b_b32_128", 32, 128, 32, 32)
case("3b_8k", 1, 8192, 24, 8)
case("3b_b4_1k", 4, 1024, 24, 8)

"""Decode attention time vs batch / context on MI355X (fused RoPE+append path, default split plan):
separates per-workgroup latency from bandwidth (us per call, HBM-resident cache)."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.ops import reference as ref  # noqa: E402
sys.path.insert(0, "scripts")


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

dev = torch.device("cuda:0")
cos, sin = ref.rope_tables(128, 8192, 500000.0, device=dev)


def run(B, H, Hkv, ctx, nparts=2, plan_ctx=None):
    nblk = (ctx + 63) // 64
    total = B * nblk * 4 + 1
    kc = torch.randn(total, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = (torch.randperm(total - 1, device=dev)[: B * nblk].int() + 1).view(B, nblk)
    pos = torch.full((B,), ctx - 1, device=dev, dtype=torch.int32)
    parts = torch.randn(nparts, B, (H + 2 * Hkv) * 128, device=dev)
    q = torch.empty(B, H, 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(q)
    ws = ops.decode_workspace(B, H, Hkv, 256, dev)
    plan = ops.decode_split_plan(B, Hkv, plan_ctx or ctx)
    us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, pos, H, Hkv, 1 / math.sqrt(128), out, workspace=ws,
                                        plan=plan, qkv_parts=parts, cos=cos, sin=sin))
    mb = B * ctx * Hkv * 128 * 2 * 2 / 1e6
    return {"B": B, "H": H, "Hkv": Hkv, "ctx": ctx, "plan": plan, "us": round(us, 2), "MB": round(mb, 1),
            "TBps": round(mb / us, 2)}


if __name__ == "__main__":
    # graphs are planned for the engine's max_model_len; short live contexts leave most splits empty
    for pc in (None, 512, 2048, 4096, 8192):
        print(json.dumps({"plan_ctx": pc, **run(32, 32, 32, 200, plan_ctx=pc)}), flush=True)
    for pc in (None, 4096, 8192):
        print(json.dumps({"plan_ctx": pc, **run(1, 24, 8, 300, plan_ctx=pc)}), flush=True)
    if len(sys.argv) > 1 and sys.argv[1] == "plans":
        sys.exit(0)
    for B in (1, 4, 8, 16, 32, 64):
        print(json.dumps(run(B, 32, 32, 200)), flush=True)
    for ctx in (64, 128, 256, 512, 1024, 2048, 4096):
        print(json.dumps(run(32, 32, 32, ctx)), flush=True)
    for ctx in (256, 512, 1024, 2100, 4096, 8192):
        print(json.dumps(run(1, 24, 8, ctx)), flush=True)

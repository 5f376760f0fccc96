"""Batch-1 residual-reduce GEMM configurations (ops.linear_rr bf16 / ops.linear_a8_rr W8A8-W4A8): every (nb, splitk,
waves, div) the kernels take for the qkv (f32 slabs) and gate_up (SiLU) projections of the BASELINE models, with the
slab count their prologue sums in the engine (the previous row-parallel projection's split-K), weights cold (a 512
MiB write before each call, as in the engine, whose per-step weights exceed the Infinity Cache).  The prologue
re-reads its residual slice once per workgroup, so the plain kernel's table pick (wide grids of narrow workgroups)
need not be the RR kernel's best.  One JSON line per shape: default pick, best config, all timings (median of 5).
Usage: sweep_rr_b1.py [shape,...]"""
import itertools
import json
import statistics as st
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
flush = torch.empty(128 << 20, device=dev)


def np_for(prev_N, prev_K, kind):  # split-K of the previous projection (o for gate_up, down for qkv) at batch 1
    if kind == "bf16":
        return ops.pick_gemm_config(1, prev_N, prev_K, "f32", kind="bf16")[1]
    return ops.pick_gemm_config(1, prev_N, prev_K, "f32", xf=True, kind="fp8a" if kind == "fp8" else "fp4a")[1]


# name: (N, K, epi, kind, previous projection (N, K))
SHAPES = {
    "3b_qkv": (5120, 3072, "f32", "bf16", (3072, 8192)), "3b_gateup": (16384, 3072, "silu", "bf16", (3072, 3072)),
    "7b_qkv": (12288, 4096, "f32", "bf16", (4096, 11008)), "7b_gateup": (22016, 4096, "silu", "bf16", (4096, 4096)),
    "7b_qkv_mx": (12288, 4096, "f32", "mxfp4", (4096, 11008)), "7b_gateup_mx": (22016, 4096, "silu", "mxfp4", (4096, 4096)),
}
names = sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1] else list(SHAPES)


def timed(fn):
    ts = []
    for _ in range(6):
        flush.fill_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    return st.median(ts[1:])


for name in names:
    N, K, epi, kind, prev = SHAPES[name]
    np_ = np_for(*prev, kind)
    g = torch.Generator(device="cpu").manual_seed(1)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16).to(dev)
    pw = ops.PackedWeight.from_dense(w, kind)
    h = torch.randn(1, K, device=dev)
    parts = torch.randn(np_, 1, K, device=dev) * 0.1
    h_out = torch.empty(1, K, device=dev)
    ss = torch.zeros(1, dtype=torch.int64, device=dev)
    a8 = kind != "bf16"
    if a8:
        nbs = (1, 2, 4, 8) if epi == "f32" else (4, 8)
        divs = (2, 4)  # fp8 chunk depth 2 / 1
    else:
        nbs = (1, 2, 4) if epi == "f32" else (2, 4)
        divs = (1, 2, 4)
    sks = (1, 2, 4, 8) if epi == "f32" else (1,)
    res = {}
    for nb, sk, wv, dv in itertools.product(nbs, sks, (4, 8), divs):
        out = (torch.empty(sk, 1, N, device=dev) if epi == "f32" else torch.empty(1, N // 2, device=dev,
                                                                                   dtype=torch.bfloat16))
        if a8:
            xo = torch.zeros(16 * N // 2, dtype=torch.uint8, device=dev) if epi == "silu" else None
            so = torch.zeros(64 * (N // 2) // 128 + 64, dtype=torch.uint8, device=dev) if epi == "silu" else None
            fn = lambda: ops.linear_a8_rr(h, parts, h_out, pw, epi, out=xo if epi == "silu" else out, out_s8=so,  # noqa
                                          ss_out=ss, eps=1e-5, splitk=sk, nb=nb, waves=wv, div=dv)
        else:
            fn = lambda: ops.linear_rr(h, parts, h_out, pw, epi, out=out, ss_out=ss, eps=1e-5, splitk=sk, nb=nb,  # noqa
                                       waves=wv, div=dv)
        try:
            fn()
            torch.cuda.synchronize()
        except RuntimeError as e:  # a configuration the kernel refuses
            res[f"{nb},{sk},{wv},{dv}"] = str(e)[:40]
            continue
        res[f"{nb},{sk},{wv},{dv}"] = round(timed(fn), 2)
    dflt = ops.rr_config(N, K, epi, kind)
    ok = {k: v for k, v in res.items() if isinstance(v, float)}
    best = min(ok, key=ok.get)
    print(json.dumps({"shape": name, "N": N, "K": K, "epi": epi, "kind": kind, "np": np_, "default": list(dflt),
                      "default_us": res.get(",".join(map(str, dflt))), "best": best, "best_us": ok[best],
                      "all": res}), flush=True)

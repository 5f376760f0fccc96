"""Prefill GEMM on MI355X: the stream-K 256^2 kernel (ops.gemm_sk, csrc/kernels/gemm_tile256.hip) vs hipBLASLt
(torch.mm on a row-major copy, measured here only as the yardstick) at the prefill shapes of the BASELINE configs:
7B qkv / o / down / gate_up at 128, 300, 1024 and 4096 rows (NL->SQL prompts, batch-1 and batch-32 bench prefill)
and the 3B's four at 2048 rows (the explain_error prompt).

Each shape runs the epilogue the engine uses: qkv bf16, gate_up SiLU(gate) * up (vendor: bf16 GEMM + the SiLU
pass), o / down accumulated into the f32 residual (vendor: addmm beta = 1 into f32).  Random operands (zero-filled
data reads high), every arm checked against an fp32 product first, arms interleaved over rounds in one process
(cdna_hip_programming.md §5.4 rule 24), median of the rounds.  Usage: bench_prefill_gemm.py [shape,shape,...]
[--shares 4,8,16] [--cold]."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


_flush = None


def timeit(fn, it=20):
    if args.cold:  # every call from cold caches: a 512 MiB write (> the 256 MiB Infinity Cache) before each, timed alone
        ts = []
        for _ in range(it // 2):
            _flush.fill_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000)
        return sorted(ts)[len(ts) // 2]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / it


SHAPES = {}
for m in (128, 300, 1024, 4096):
    SHAPES[f"7b_qkv_m{m}"] = (m, 12288, 4096, "bf16")
    SHAPES[f"7b_o_m{m}"] = (m, 4096, 4096, "res")
    SHAPES[f"7b_gateup_m{m}"] = (m, 22016, 4096, "silu")
    SHAPES[f"7b_down_m{m}"] = (m, 4096, 11008, "res")
SHAPES.update({"3b_qkv_m2048": (2048, 5120, 3072, "bf16"), "3b_o_m2048": (2048, 3072, 3072, "res"),
               "3b_gateup_m2048": (2048, 16384, 3072, "silu"), "3b_down_m2048": (2048, 3072, 8192, "res")})
# --grid: every model projection at M = 128 .. 4096 (the tuning sweep behind ops/gemm_sk_tuning.json)
GRID = {}
for m in (128, 256, 300, 512, 1024, 2048, 4096):  # 300: the NL->SQL prompt length (3 row tiles of 128, one ragged)
    for mod, d, nq, f in (("7b", 4096, 12288, 11008), ("3b", 3072, 5120, 8192)):
        GRID[f"{mod}_qkv_m{m}"] = (m, nq, d, "bf16")
        GRID[f"{mod}_o_m{m}"] = (m, d, d, "res")
        GRID[f"{mod}_gateup_m{m}"] = (m, 2 * f, d, "silu")
        GRID[f"{mod}_down_m{m}"] = (m, d, f, "res")

ap = argparse.ArgumentParser()
ap.add_argument("shapes", nargs="?", default="")
ap.add_argument("--shares", default=str(ops.SK_MIN_SHARE))
ap.add_argument("--cfgs", default="-2", help="tile configurations (ops.SK_CFGS index, +8 whole tiles only; -1 the "
                "kernel's cost model, -2 the measured table the engine uses)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--epls", default="1", help="epilogue modes to compare (0 direct, 1 through LDS)")
ap.add_argument("--nbufs", default="3", help="K-tile buffer counts to compare (3: three where they fit, 2: two)")
ap.add_argument("--grid", action="store_true")
ap.add_argument("--no-vendor", action="store_true")
ap.add_argument("--cold", action="store_true", help="time each call alone after a 512 MiB cache-flushing write (the "
                "engine's case: a layer's weights come from HBM, not from the Infinity Cache of the previous call)")
args = ap.parse_args()
if args.cold:
    _flush = torch.empty(128 << 20, device=dev)
src = GRID if args.grid else SHAPES
shapes = {k: v for k, v in src.items() if not args.shapes or k in args.shapes.split(",")}
shares = [int(s) for s in args.shares.split(",")]
cfgs = [int(c) for c in args.cfgs.split(",")]
epls = [int(c) for c in args.epls.split(",")]
nbufs = [int(c) for c in args.nbufs.split(",")]
e = ops.ext()
for name, (M, N, K, epi) in shapes.items():
    torch.manual_seed(0)
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    pw = ops.PackedWeight.from_dense(w)
    wt = w.t()
    ref = x.float() @ w.float().t()
    h0 = torch.randn(M, N, device=dev)
    if epi == "silu":
        r3 = ref.view(M, N // 32, 2, 16)
        ref = (torch.nn.functional.silu(r3[:, :, 0]) * r3[:, :, 1]).reshape(M, N // 2)
        out = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
        y16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    elif epi == "res":
        ref = ref + h0
        out = h0.clone()
    else:
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    arms = {}
    for cf in cfgs:
        if epi == "silu" and cf >= 0 and not ops.sk_cfg_pairs(cf):
            continue  # SiLU pairs need an even n-block count per wave
        for sh in shares:
            for ep in epls:
                for nbf in nbufs:
                    tag = ("table" if cf == -2 else "auto") if cf < 0 else ops.sk_cfg_tag(cf)
                    arm_name = (f"sk_{tag}_s{sh}" + ("" if len(nbufs) == 1 else f"_b{nbf}") +
                                ("" if len(epls) == 1 else f"_e{ep}"))

                    def arm(sh=sh, cf=cf, ep=ep, nbf=nbf):
                        e.gemm_sk_epilogue(ep)
                        e.gemm_sk_nbuf(nbf)
                        ops.gemm_sk(x, pw.data, N, out, epi, min_share=sh, cfg=None if cf == -2 else cf)
                    arms[arm_name] = arm
    if epi == "silu":
        def blas():
            torch.mm(x, wt, out=y16)
            e.silu_bf16(y16, out)
    elif epi == "res":
        def blas():
            torch.addmm(out, x, wt, out_dtype=torch.float32, out=out)
    else:
        def blas():
            torch.mm(x, wt, out=out)
    if not args.no_vendor:
        arms["hipblaslt"] = blas
    res = {"shape": name, "M": M, "N": N, "K": K, "epi": epi}
    flops = 2.0 * M * N * K
    for an, fn in arms.items():
        if epi == "res":
            out.copy_(h0)
        fn()
        torch.cuda.synchronize()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        res[an] = {"rel_err": float(f"{err:.2e}")}
        if an.startswith("sk") and not args.grid:
            # every call leaves the tickets zero and is bitwise reproducible
            first = out.clone()
            if epi == "res":
                out.copy_(h0)
            fn()
            torch.cuda.synchronize()
            res[an]["repeat_bitwise"] = bool(torch.equal(first, out))
    times = {an: [] for an in arms}
    for _ in range(args.rounds):
        for an, fn in arms.items():
            fn()
            times[an].append(timeit(fn))
    for an in arms:
        us = sorted(times[an])[len(times[an]) // 2]
        res[an].update({"us": round(us, 1), "TF": round(flops / us / 1e6, 1)})
    print(json.dumps(res), flush=True)
    del x, w, pw, out, ref, h0
    torch.cuda.empty_cache()

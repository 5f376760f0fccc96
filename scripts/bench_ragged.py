"""Ragged decode-GEMM grids (gemm.hip: nb not dividing the n-blocks -> ceil(NBtot / nb) workgroups, blocks dealt
evenly) vs the divisible widths, at the decode shapes whose divisible grids under- or over-fill 256 CUs
(7B gate_up: 1376 n-blocks = 172 workgroups at nb 8, 344 at nb 4).  Numerics vs fp32 first, then us per call
with weights rotating over > 600 MiB (HBM-streamed), median of 3 x 40; activations fragment-major for M > 16
(as the decode step runs them).  Usage: python scripts/bench_ragged.py [M,M,..] [shape,shape,..]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"7b_gateup": (22016, 4096, "silu"), "7b_qkv": (12288, 4096, "f32"), "7b_head": (32000, 4096, "f32"),
          "3b_gateup": (16384, 3072, "silu"), "3b_qkv": (5120, 3072, "f32"), "7b_down": (4096, 11008, "f32"),
          "7b_o": (4096, 4096, "f32"), "3b_down": (3072, 8192, "f32"), "3b_o": (3072, 3072, "f32")}
Ms = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 32]
if len(sys.argv) > 2:
    SHAPES = {k: v for k, v in SHAPES.items() if k in sys.argv[2].split(",")}
KIND = sys.argv[3] if len(sys.argv) > 3 else "bf16"  # bf16 | mxfp4 (gemm_fp4.hip) | fp8a (W8A8, gemm_fp8a.hip)
WKIND = "fp8" if KIND == "fp8a" else KIND


def run(x, w, M, epi, out, nb, sk, wv, dv, xf):
    if KIND == "fp8a":  # x = (x8, sx) in the xf8 layout; div = chunk depth selector
        return ops.linear_a8(x[0], x[1], M, w, epi, out=out, splitk=sk, nb=nb, waves=wv, div=dv, xfo=xf)
    if xf:
        return ops.linear_xf(x, M, w, epi, out=out, splitk=sk, nb=nb, waves=wv, div=dv)
    return ops.linear(x, w, epi, out=out, splitk=sk, nb=nb, waves=wv, div=dv)


for name, (N, K, epi) in SHAPES.items():
    nbytes = {"bf16": N * K * 2, "mxfp4": N * K * 17 // 32, "fp8a": N * K}[KIND]
    ncopy = max(2, (600 << 20) // nbytes + 1)
    dense = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
    ws = [ops.PackedWeight.from_dense(d, WKIND) for d in dense]
    if KIND != "bf16":  # the oracle multiplies the weights the kernel sees
        dense[0] = ws[0].dense()
    for M in Ms:
        xf = 16 < M <= 64
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xin = ops.to_xfrag(x) if xf else x
        if KIND == "fp8a":
            x8, sx8 = ops.quantize_xf8(x)
            xin = (x8, sx8)
            x = (ops.from_xf8(x8, M, K).view(torch.float8_e4m3fn).float() * sx8[:M, None])
        yr = x.float() @ dense[0].float().t()
        if epi == "silu":
            y3 = yr.view(M, N // 32, 2, 16)
            yr = (torch.nn.functional.silu(y3[:, :, 0]) * y3[:, :, 1]).reshape(M, N // 2)
        pick = ops.pick_gemm_config(M, N, K, epi, xf=True, kind=KIND) if KIND == "fp8a" else \
            ops.pick_gemm_config(M, N, K, epi, xf=xf, kind=KIND)
        cands = {tuple(pick)}
        for nb in ((4, 6, 8) if KIND == "bf16" else (1, 2, 4, 6, 8)):
            for dv in ((1, 2) if KIND == "bf16" else (4,) if KIND == "mxfp4" else (2, 4)):
                for sk in ((1,) if epi == "silu" else (1, 2, 4, 8)):
                    for wv in ((4,) if KIND == "bf16" else (4, 8)):  # (fp8a: div 2 = depth 2, 4 = depth 1)
                        cands.add((nb, sk, wv, dv))
        for nb, sk, wv, dv in sorted(cands):
            if (epi == "silu" and nb % 2) or (M > 32 and nb > 2) or (nb == 6 and M <= 16):
                continue  # (nb 6 is instantiated for two row tiles only; one row tile would fall back to nb 2)
            if epi == "silu":
                out = torch.empty(ops.xfrag_tiles(M) * 16 * (N // 2) if xf else M * N // 2, device=dev,
                                  dtype=torch.bfloat16)
                o = out if xf else out.view(M, N // 2)
            else:
                o = torch.empty(sk, M, N, device=dev)
            y = run(xin, ws[0], M, epi, o, nb, sk, wv, dv, xf)
            got = (ops.from_xfrag(y, M, N // 2) if xf else y) if epi == "silu" else y.sum(0)
            err = ((got.float() - yr).norm() / yr.norm()).item()
            assert err < 1e-2, (name, M, nb, sk, err)
            for i in range(3):
                run(xin, ws[i % ncopy], M, epi, o, nb, sk, wv, dv, xf)
            torch.cuda.synchronize()
            reps = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(40):
                    run(xin, ws[i % ncopy], M, epi, o, nb, sk, wv, dv, xf)
                e1.record()
                torch.cuda.synchronize()
                reps.append(e0.elapsed_time(e1) * 1000 / 40)
            us = sorted(reps)[1]
            nbt = N // 16
            print(json.dumps(dict(shape=name, kind=KIND, M=M, nb=nb, splitk=sk, waves=wv, div=dv, ragged=bool(nbt % nb),
                                  wgs=-(-nbt // nb) * sk, us=round(us, 2), TBps=round(nbytes / us / 1e6, 3),
                                  picked=list(pick) == [nb, sk, wv, dv], err=round(err, 5))), flush=True)
    del ws, dense
    torch.cuda.empty_cache()

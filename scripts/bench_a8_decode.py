"""W8A8 / W4A8 decode GEMM (e4m3 activations on the block-scaled fp8 MFMA, csrc/kernels/gemm_fp8a.hip) vs the
16-bit-activation decode GEMM it replaces (W8A16 gemm_fp8.hip / W4A16 gemm_fp4.hip), per projection of the 7B and
the 3B, at the decode buckets; sweep over (nb, splitk, waves, depth).  Activations as the engine hands them over:
qkv / gate_up per-row f32 scales (the RMSNorm launch), o per-(row, head) E8M0 (the attention), down per-(row, 32)
E8M0 (the SiLU epilogue); 'silu8' = gate_up writing the down input as e4m3.  Weights rotate over > 600 MiB so they
stream from HBM.  Each line carries a "tune" entry (key "NxK:epi:b<M>:fp8a|fp4a", 4th field = chunk depth as 'div':
2 -> depth 2) when the sweep beats the default pick by > 3 %; scripts/merge_tuning.py folds them in.

    python scripts/bench_a8_decode.py fp8|mxfp4 [Ms]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
KIND = sys.argv[1] if len(sys.argv) > 1 else "fp8"
AK = "fp8a" if KIND == "fp8" else "fp4a"
Ms = [int(a) for a in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 4, 16, 32, 64]
# name: (N, K, epi, activation scaling)
SHAPES = {"7b_qkv": (12288, 4096, "f32", "row"), "7b_o": (4096, 4096, "f32", "b128"),
          "7b_gateup": (22016, 4096, "silu", "row"), "7b_gateup8": (22016, 4096, "silu8", "row"),
          "7b_down": (4096, 11008, "f32", "b32"),
          "3b_qkv": (5120, 3072, "f32", "row"), "3b_o": (3072, 3072, "f32", "b128"),
          "3b_gateup8": (16384, 3072, "silu8", "row"), "3b_down": (3072, 8192, "f32", "b32")}


def timeit(fn, it=30):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    reps = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(it):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        reps.append(e0.elapsed_time(e1) * 1000 / it)
    return sorted(reps)[1]


for name, (N, K, epi, scal) in SHAPES.items():
    ncopy = max(2, (600 << 20) // (N * K // (1 if KIND == "fp8" else 2)) + 1)
    ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), KIND)
          for _ in range(ncopy)]
    e16 = "silu" if epi == "silu8" else epi
    for M in Ms:
        mt = ops.xfrag_tiles(M)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xf = ops.to_xfrag(x)
        if scal == "row":
            x8, sx = ops.quantize_xf8(x)
            s8 = None
        else:
            x8, s8 = ops.quantize_xf8_blocks(x, 128 if scal == "b128" else 32)
            sx = None
        o8 = torch.zeros(mt * 16 * N // 2, device=dev, dtype=torch.uint8) if epi == "silu8" else None
        os8 = torch.zeros(mt * 64 * max(1, N // 2 // 128), device=dev, dtype=torch.uint8) if epi == "silu8" else None

        def out(sk):
            if epi == "f32":
                return torch.empty(sk, M, N, device=dev)
            if epi == "silu8":
                return o8
            return torch.empty(mt * 16 * (N // 2), device=dev, dtype=torch.bfloat16)

        def run_a8(o, **kw):
            return lambda i: ops.linear_a8(x8, sx, M, ws[i % ncopy], "silu" if epi == "silu8" else epi, out=o, s8=s8,
                                           out_s8=os8, **kw)

        w16 = ops.pick_gemm_config(M, N, K, e16, xf=True, kind=KIND)
        o16 = torch.empty(w16[1], M, N, device=dev) if e16 == "f32" else torch.empty(
            mt * 16 * (N // 2), device=dev, dtype=torch.bfloat16)
        res = {"shape": name, "kind": KIND, "M": M, "epi": epi, "a16_cfg": list(w16),
               "a16_us": round(timeit(lambda i: ops.linear_xf(xf, M, ws[i % ncopy], e16, out=o16)), 2)}
        pick = ops.pick_gemm_config(M, N, K, epi, xf=True, kind=AK)
        res["a8_pick"] = list(pick)
        res["a8_pick_us"] = round(timeit(run_a8(out(pick[1]))), 2)
        best = None
        for waves in (4, 8):
            for depth in (1, 2):
                for nb in (1, 2, 4, 6, 8):
                    if (epi != "silu8" and (N // 16) % nb) or (epi.startswith("silu") and nb % 2):
                        continue
                    if epi == "silu8" and (nb % 4 or (N // 16) % nb):
                        continue
                    if M > 32 and nb > 2 and not (epi == "silu8" and nb == 4):
                        continue
                    if nb >= 6 and (waves != 4 or depth != 1 or M > 32 or (nb == 6 and M <= 16)):
                        continue  # (nb 6 is instantiated for the two-row-tile kernels only)
                    for sk in ((1, 2, 4, 8) if epi == "f32" else (1,)):
                        kb = K // 128
                        kbps = (kb + sk - 1) // sk
                        if kbps < 2 or (kb + kbps - 1) // kbps != sk:
                            continue
                        dv = 2 if depth == 2 else 4
                        us = timeit(run_a8(out(sk), splitk=sk, nb=nb, waves=waves, div=dv))
                        if best is None or us < best[1]:
                            best = ((nb, sk, waves, dv), us)
        res["a8_best"], res["a8_best_us"] = list(best[0]), round(best[1], 2)
        res["GBps_best"] = round(N * K / (1 if KIND == "fp8" else 2) / best[1] / 1e3, 1)
        if best[1] < 0.97 * res["a8_pick_us"] and M in (1, 2, 4, 8, 16, 32, 64):
            nb, sk, wv, dv = best[0]
            res["tune"] = {f"{N}x{K}:{epi}:b{M}:{AK}": {"nb": nb, "splitk": sk, "waves": wv, "div": dv,
                                                       "us": round(best[1], 2),
                                                       "note": f"scripts/bench_a8_decode.py: pick {res['a8_pick_us']} us"}}
        print(json.dumps(res), flush=True)
    del ws
    torch.cuda.empty_cache()

"""Decode GEMM at the batch buckets between the tuned M = 1 / M = 32 points: the config ops picks from the
tuning table vs the best of a sweep over (nb, splitk, waves, div), per shape and M (us per call, weights
rotating over > 600 MiB so they stream from HBM).  Prints one JSON line per (shape, M)."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"7b_qkv": (12288, 4096, "f32"), "7b_o": (4096, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"),
          "7b_down": (4096, 11008, "f32"), "3b_qkv": (5120, 3072, "f32"), "3b_gateup": (16384, 3072, "silu"),
          "3b_down": (3072, 8192, "f32"), "3b_o": (3072, 3072, "f32")}
Ms = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4, 8, 16, 24, 48, 64]
KIND = sys.argv[2] if len(sys.argv) > 2 else "bf16"  # fp8: OCP e4m3 weights (the fp8 kernel has no waves/div knobs)
if len(sys.argv) > 3:  # shape subset
    SHAPES = {k: v for k, v in SHAPES.items() if k in sys.argv[3].split(",")}
NBS = tuple(int(a) for a in os.environ.get("LSA_SWEEP_NBS", "1,2,4").split(","))


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


for name, (N, K, epi) in SHAPES.items():
    nbytes = N * K * 2
    ncopy = max(2, (600 << 20) // nbytes + 1)
    nbytes = nbytes // 2 if KIND == "fp8" else nbytes
    ncopy = max(2, (600 << 20) // nbytes + 1)
    ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), KIND)
          for _ in range(ncopy)]
    for M in Ms:
        xf = M > 16 and M <= 64
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xfr = ops.to_xfrag(x) if xf else None

        def call(cfg):
            nb, sk, waves, dv = cfg
            o = (torch.empty(sk, M, N, device=dev) if epi == "f32" else
                 torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16))
            if xf:
                return lambda i: ops.linear_xf(xfr, M, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb, waves=waves, div=dv)
            return lambda i: ops.linear(x, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb, waves=waves, div=dv)

        picked = ops.pick_gemm_config(M, N, K, epi, xf=xf, kind=KIND)
        res = {"shape": name, "M": M, "xf": xf, "kind": KIND, "picked": list(picked), "picked_us": round(timeit(call(picked)), 2)}
        best = None
        for waves, dv in (((4, 1), (4, 2), (4, 4), (8, 2)) if KIND == "bf16" else ((4, 4),)):
            for nb in NBS:
                if (N // 16) % nb or (epi == "silu" and nb % 2) or (M > 32 and nb > 2) or (nb == 6 and M <= 16):
                    continue
                if nb >= 6 and (waves, dv) not in ((4, 1), (4, 2)):  # wide n-groups: 4 waves, div 1 | 2 only
                    continue
                if waves == 16 and (M > 16 or nb > 2):  # the 16-wave kernel: one row tile, nb <= 2
                    continue
                for sk in ((1, 2, 4, 8) if epi == "f32" else (1,)):
                    if K // 32 // sk < 8:
                        continue
                    us = timeit(call((nb, sk, waves, dv)))
                    if best is None or us < best[1]:
                        best = ((nb, sk, waves, dv), us)
        # re-time the pick after the sweep (the first timing of a shape can include one-time warm-up)
        res["picked_us"] = round(min(res["picked_us"], timeit(call(picked))), 2)
        res["best"] = list(best[0])
        res["best_us"] = round(best[1], 2)
        print(json.dumps(res), flush=True)
    del ws
    torch.cuda.empty_cache()

"""W8A8 decode GEMM (fp8 activations + weights on the fp8 MFMA, csrc/kernels/gemm_fp8a.hip) vs the W8A16
decode GEMM it replaces for the qkv / gate_up projections, at the fragment-major decode buckets; sweep over
(nb, splitk, waves, depth).  Weights rotate over > 600 MiB so they stream from HBM.  Each line carries a
"tune" entry (key "NxK:epi:b<M>:fp8a", 4th field = chunk depth as 'div': 2 -> depth 2) when the sweep beats the
default pick by > 3 %; scripts/merge_tuning.py folds them in.

    python scripts/bench_fp8a_decode.py [Ms]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"7b_qkv": (12288, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"),
          "3b_qkv": (5120, 3072, "f32"), "3b_gateup": (16384, 3072, "silu")}
Ms = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [20, 32, 64]


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
    ncopy = max(2, (600 << 20) // (N * K) + 1)
    ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), "fp8")
          for _ in range(ncopy)]
    for M in Ms:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xf = ops.to_xfrag(x)
        x8, sx = ops.quantize_xf8(x)

        def out(sk):
            if epi == "f32":
                return torch.empty(sk, M, N, device=dev)
            return torch.empty(ops.xfrag_tiles(M) * 16 * (N // 2), device=dev, dtype=torch.bfloat16)

        w16 = ops.pick_gemm_config(M, N, K, epi, xf=True, kind="fp8")
        o16 = out(w16[1])
        res = {"shape": name, "M": M, "epi": epi, "w8a16_cfg": list(w16),
               "w8a16_us": round(timeit(lambda i: ops.linear_xf(xf, M, ws[i % ncopy], epi, out=o16)), 2)}
        pick = ops.pick_gemm_config(M, N, K, epi, xf=True, kind="fp8a")
        op = out(pick[1])
        res["w8a8_pick"] = list(pick)
        res["w8a8_pick_us"] = round(timeit(lambda i: ops.linear_a8(x8, sx, M, ws[i % ncopy], epi, out=op)), 2)
        best = None
        for waves in (4, 8):
            for depth in (1, 2):
                for nb in (1, 2, 4, 6, 8):
                    if (N // 16) % nb or (epi == "silu" and nb % 2) or (M > 32 and nb > 2):
                        continue
                    if nb >= 6 and (waves != 4 or depth != 1 or not 16 < M <= 32):
                        continue
                    for sk in ((1, 2, 4, 8) if epi == "f32" else (1,)):
                        kb = K // 128
                        kbps = (kb + sk - 1) // sk
                        if kbps < 2 or (kb + kbps - 1) // kbps != sk:
                            continue
                        o = out(sk)
                        dv = 2 if depth == 2 else 4
                        us = timeit(lambda i: ops.linear_a8(x8, sx, M, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb,
                                                            waves=waves, div=dv))
                        if best is None or us < best[1]:
                            best = ((nb, sk, waves, dv), us)
        res["w8a8_best"], res["w8a8_best_us"] = list(best[0]), round(best[1], 2)
        res["GBps_best"] = round(N * K / best[1] / 1e3, 1)
        if best[1] < 0.97 * res["w8a8_pick_us"] and M in (1, 2, 4, 8, 16, 32, 64):
            nb, sk, wv, dv = best[0]
            res["tune"] = {f"{N}x{K}:{epi}:b{M}:fp8a": {"nb": nb, "splitk": sk, "waves": wv, "div": dv,
                                                          "us": round(best[1], 2),
                                                          "note": f"scripts/bench_fp8a_decode.py: pick {res['w8a8_pick_us']} us"}}
        print(json.dumps(res), flush=True)
    del ws
    torch.cuda.empty_cache()

"""MXFP4 W4A16 decode GEMM (csrc/kernels/gemm_fp4.hip) over (nb, splitk, waves) at the 7B / 3B decode shapes:
us per call and the weight stream's rate (e2m1 + scale bytes).  Weights rotate over > 600 MiB so they stream from
HBM.  One JSON line per (shape, M) with the best config and a ready "tune" entry ("NxK:epi:b<M>:fp4");
scripts/merge_tuning.py folds them into ops/gemm_tuning.json.

    python scripts/bench_fp4_decode.py [Ms]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"7b_qkv": (12288, 4096, "f32"), "7b_o": (4096, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"),
          "7b_down": (4096, 11008, "f32"), "7b_lm_head": (32000, 4096, "f32"), "3b_qkv": (5120, 3072, "f32"),
          "3b_o": (3072, 3072, "f32"), "3b_gateup": (16384, 3072, "silu"), "3b_down": (3072, 8192, "f32")}
Ms = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 32]


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
    nbytes = N * K // 2 + (N // 16) * ((K // 128 + 3) // 4) * 256
    ncopy = max(2, (600 << 20) // nbytes + 1)
    ws = [ops.PackedWeight.from_dense(torch.randn(N, K, device=dev) * 0.02, "mxfp4") for _ in range(ncopy)]
    for M in Ms:
        xf = 16 < M <= 64
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xin = ops.to_xfrag(x) if xf else x
        pick = ops.pick_gemm_config(M, N, K, epi, xf=xf, kind="mxfp4")
        res = {"shape": name, "M": M, "xf": xf, "pick": list(pick[:3])}
        best = None
        for nb in (1, 2, 4, 8):
            if (epi == "silu" and nb < 2) or (N // 16) % nb or (M > 32 and nb > 2) or (nb == 8 and M > 32):
                continue
            for sk in ((1, 2, 4, 8) if epi == "f32" else (1,)):
                for waves in (4, 8):
                    out = (torch.empty(sk, M, N, device=dev) if epi == "f32" else
                           torch.empty(ops.xfrag_tiles(M) * 16 * N // 2 if xf else M * N // 2, device=dev,
                                       dtype=torch.bfloat16))

                    def run(i, nb=nb, sk=sk, waves=waves, out=out):
                        if xf:
                            ops.linear_xf(xin, M, ws[i % ncopy], epi, out=out, splitk=sk, nb=nb, waves=waves)
                        else:
                            ops.linear(xin, ws[i % ncopy], epi, out=out, splitk=sk, nb=nb, waves=waves)

                    us = timeit(run)
                    if best is None or us < best[0]:
                        best = (us, nb, sk, waves)
                    if (nb, sk, waves) == tuple(pick[:3]):
                        res["pick_us"] = round(us, 2)
        us, nb, sk, waves = best
        res.update(best_us=round(us, 2), best=[nb, sk, waves], TBps=round(nbytes / us / 1e6, 2))
        b = 1
        while b < M:
            b *= 2
        res["tune"] = {f"{N}x{K}:{epi}:b{b}:fp4": {"nb": nb, "splitk": sk, "waves": waves, "us": round(us, 2),
                                                    "note": "scripts/bench_fp4_decode.py"}}
        print(json.dumps(res), flush=True)
    del ws
    torch.cuda.empty_cache()

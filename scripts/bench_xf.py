"""Row-major vs fragment-major activations in the decode GEMM (M = 32 / 1, 7B and 3B shapes):
best config of each over (nb, splitk, waves, div).  Weights rotate over > 600 MiB of copies."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"7b_qkv": (12288, 4096, "f32"), "7b_o": (4096, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"),
          "7b_down": (4096, 11008, "f32"), "3b_qkv": (5120, 3072, "f32"), "3b_gateup": (16384, 3072, "silu"),
          "3b_down": (3072, 8192, "f32"), "3b_o": (3072, 3072, "f32")}
Ms = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [32]
if len(sys.argv) > 2:
    SHAPES = {k: v for k, v in SHAPES.items() if k in sys.argv[2].split(",")}
MODES = sys.argv[3].split(",") if len(sys.argv) > 3 else ["row", "xf"]


def timeit(fn, it=40):
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


out_rows = []
for name, (N, K, epi) in SHAPES.items():
    nbytes = N * K * 2
    ncopy = max(2, (600 << 20) // nbytes + 1)
    ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(ncopy)]
    for M in Ms:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xf = ops.to_xfrag(x)
        best = {}
        for mode in MODES:
            for waves, dv in ((4, 1), (4, 2), (8, 2), (4, 4), (8, 1)):
                for nb in (1, 2, 4):
                    if (N // 16) % nb or (epi == "silu" and nb == 1) or (M > 32 and nb > 2):
                        continue
                    for sk in ((1, 2, 4, 8) if epi == "f32" else (1,)):
                        if K // 32 // sk < 8:
                            continue
                        o = (torch.empty(sk, M, N, device=dev) if epi == "f32" else
                             torch.empty(M, N // 2 if epi == "silu" else N, device=dev, dtype=torch.bfloat16))
                        if mode == "row":
                            f = lambda i: ops.linear(x, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb, waves=waves, div=dv)  # noqa: E731
                        else:
                            f = lambda i: ops.linear_xf(xf, M, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb,  # noqa: E731
                                                        waves=waves, div=dv)
                        us = timeit(f)
                        r = dict(shape=name, M=M, mode=mode, nb=nb, splitk=sk, waves=waves, div=dv, us=round(us, 2),
                                 TBps=round(nbytes / us / 1e6, 3))
                        out_rows.append(r)
                        if mode not in best or us < best[mode]["us"]:
                            best[mode] = r
        for mode in MODES:
            if mode in best:
                print("BEST", json.dumps(best[mode]), flush=True)
    del ws
    torch.cuda.empty_cache()
json.dump(out_rows, open("gpurun_out/xf_sweep.json", "w"), indent=0)

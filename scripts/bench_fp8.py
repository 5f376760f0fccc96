"""fp8-weight decode GEMM sweep (nb x splitk) at M = 1 and 32 (fragment-major activations at 32) for the
7B shapes; writes the best configs as ':fp8' tuning entries to gpurun_out/fp8_tuning.json."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"7b_qkv": (12288, 4096, "f32"), "7b_o": (4096, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"),
          "7b_down": (4096, 11008, "f32"), "7b_head": (32000, 4096, "f32")}


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


table = {}
for name, (N, K, epi) in SHAPES.items():
    nbytes = N * K
    ncopy = max(2, (600 << 20) // nbytes + 1)
    ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), kind="fp8")
          for _ in range(ncopy)]
    for M in (1, 32):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xf = ops.to_xfrag(x)
        best = None
        for nb in (1, 2, 4):
            if (N // 16) % nb or (epi == "silu" and nb == 1):
                continue
            for sk in ((1, 2, 4, 8) if epi == "f32" else (1,)):
                if K // 64 // sk < 4:
                    continue
                if epi == "f32":
                    o = torch.empty(sk, M, N, device=dev)
                else:
                    o = torch.empty(max(M, 16) * (N // 2 if epi == "silu" else N) * (2 if M > 16 else 1),
                                    device=dev, dtype=torch.bfloat16)
                if M > 16:
                    f = lambda i: ops.linear_xf(xf, M, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb)  # noqa: E731
                else:
                    oo = o if epi == "f32" else o[: M * (N // 2 if epi == "silu" else N)].view(M, -1)
                    f = lambda i: ops.linear(x, ws[i % ncopy], epi, out=oo, splitk=sk, nb=nb)  # noqa: E731
                us = timeit(f)
                r = dict(shape=name, M=M, nb=nb, splitk=sk, us=round(us, 2), TBps=round(nbytes / us / 1e6, 3))
                if best is None or us < best["us"]:
                    best = r
        print("BEST", json.dumps(best), flush=True)
        key = f"{N}x{K}:{epi}:{'s' if M <= 16 else 'm'}:fp8"
        table[key] = {"nb": best["nb"], "splitk": best["splitk"], "us": best["us"], "waves": 4, "div": 4}
    del ws
    torch.cuda.empty_cache()
json.dump(table, open("gpurun_out/fp8_tuning.json", "w"), indent=1, sort_keys=True)

"""Cost of the fused residual+RMSNorm GEMM tail vs GEMM + separate add_rmsnorm kernel (decode shapes).
Weights rotate over > 600 MiB so every GEMM streams from HBM."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


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


for name, (N, K) in {"7b_o": (4096, 4096), "7b_down": (4096, 11008), "3b_o": (3072, 3072),
                     "3b_down": (3072, 8192)}.items():
    ncopy = max(2, (600 << 20) // (N * K * 2) + 1)
    ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(ncopy)]
    nw = torch.ones(N, device=dev, dtype=torch.bfloat16)
    ctr = torch.zeros(2, device=dev, dtype=torch.int32)
    for M in (1, 32):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        h = torch.randn(M, N, device=dev)
        xn = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        nb, sk, wv, dv = ops.pick_gemm_config(M, N, K, "f32")
        out = torch.empty(sk, M, N, device=dev)
        r = dict(shape=name, M=M, cfg=[nb, sk, wv, dv])
        r["gemm"] = timeit(lambda i: ops.linear(x, ws[i % ncopy], "f32", out=out, splitk=sk))
        r["norm"] = timeit(lambda i: ops.add_rmsnorm(h, nw, 1e-5, xn, parts=out))
        r["gemm+norm"] = timeit(lambda i: (ops.linear(x, ws[i % ncopy], "f32", out=out, splitk=sk),
                                           ops.add_rmsnorm(h, nw, 1e-5, xn, parts=out)))
        r["fused"] = timeit(lambda i: ops.linear_norm(x, M, ws[i % ncopy], out, h, nw, 1e-5, xn, ctr, splitk=sk))
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    del ws
    torch.cuda.empty_cache()

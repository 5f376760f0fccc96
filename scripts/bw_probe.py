"""HBM ceiling probe on the GPU: streaming-read bandwidth (torch sum / copy) vs hipBLASLt
(torch.matmul) vs our decode GEMM at the 7B decode shapes.  Weights rotate over > 600 MiB of copies
so every call streams from HBM.  Prints one JSON line per measurement."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, it=30):
    for _ in range(3):
        fn(0)
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


big = torch.empty(1 << 30, dtype=torch.bfloat16, device=dev).normal_()  # 2 GiB
us = timeit(lambda i: big.sum(dtype=torch.float32), 10)
print(json.dumps(dict(probe="torch_sum_2GiB", us=round(us, 1), TBps=round(big.numel() * 2 / us / 1e6, 3))))
dst = torch.empty_like(big)
us = timeit(lambda i: dst.copy_(big), 10)
print(json.dumps(dict(probe="torch_copy_2GiB_rw", us=round(us, 1), TBps=round(big.numel() * 4 / us / 1e6, 3))))
del big, dst
torch.cuda.empty_cache()

for name, (N, K, epi) in {"7b_qkv": (12288, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"),
                          "7b_down": (4096, 11008, "f32"), "7b_o": (4096, 4096, "f32")}.items():
    nbytes = N * K * 2
    ncopy = max(2, (600 << 20) // nbytes + 1)
    dense = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
    packed = [ops.PackedWeight.from_dense(w) for w in dense]
    for M in (1, 32):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        us = timeit(lambda i: torch.matmul(x, dense[i % ncopy].t()))
        print(json.dumps(dict(probe="hipblaslt_matmul", shape=name, M=M, us=round(us, 2), TBps=round(nbytes / us / 1e6, 3))))
        nb, sk, wv, dv = ops.pick_gemm_config(M, N, K, epi)
        cols = N // 2 if epi == "silu" else N
        out = torch.empty((sk, M, N) if epi == "f32" else (M, cols), device=dev,
                          dtype=torch.float32 if epi == "f32" else torch.bfloat16)
        us = timeit(lambda i: ops.linear(x, packed[i % ncopy], epi, out=out, splitk=sk, nb=nb, waves=wv, div=dv))
        print(json.dumps(dict(probe="lsa_linear", shape=name, M=M, cfg=[nb, sk, wv, dv], us=round(us, 2),
                              TBps=round(nbytes / us / 1e6, 3))))
    del dense, packed
    torch.cuda.empty_cache()

"""Run one stream-K prefill GEMM configuration back to back (for rocprofv3 --pmc passes): shape M N K epi cfg [iters].
Random operands.  Example: probe_gemm_sk.py 4096 4096 4096 bf16 0 50"""
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

M, N, K, epi, cfg = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5])
it = int(sys.argv[6]) if len(sys.argv) > 6 else 50
dev = torch.device("cuda:0")
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
pw = ops.PackedWeight.from_dense(w)
out = torch.zeros(M, N // 2 if epi == "silu" else N, device=dev,
                  dtype=torch.float32 if epi in ("f32", "res") else torch.bfloat16)
for _ in range(it):
    ops.gemm_sk(x, pw.data, N, out, epi, cfg=cfg)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    ops.gemm_sk(x, pw.data, N, out, epi, cfg=cfg)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / it
print(f"{M}x{N}x{K} {epi} cfg {cfg}: {us:.1f} us, {2.0 * M * N * K / us / 1e6:.0f} TF")

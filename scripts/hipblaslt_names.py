"""Runs the vendor library (torch.mm -> hipBLASLt) on the prefill GEMM shapes of scripts/bench_prefill_gemm.py so a
rocprofv3 --kernel-trace --stats pass records which kernel (macro tile, MFMA, workgroup shape) it picks per shape:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_blas -o run -- python3 scripts/hipblaslt_names.py
"""
import torch

SHAPES = [(4096, 12288, 4096), (4096, 4096, 4096), (4096, 4096, 11008), (2048, 5120, 3072), (2048, 3072, 8192),
          (300, 12288, 4096), (8192, 8192, 8192)]
dev = torch.device("cuda:0")
for M, N, K in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(3):
        torch.mm(a, b.t())
    torch.cuda.synchronize()
    print(M, N, K, flush=True)

"""Minimal repro for the round-1 `rocprofv3 --pmc` SIGSEGV (gpurun_out/pmc_b32.log: inside the first
fragment-major skinny GEMM launch, launch_skinny_t<2,2,1> <- lsa_gemm_cfg <- gemm_xf).

    python scripts/pmc_repro.py row|xf [M]

Runs the 7B qkv decode GEMM (N 12288, K 4096, f32 split-K slabs) 20 times with row-major (row) or
fragment-major (xf) activations at M rows."""
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "xf"
M = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda:0")
N, K = 12288, 4096
w = ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16))
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
xf = ops.to_xfrag(x)
o = torch.empty(2, M, N, device=dev)
for i in range(20):
    if mode == "xf":
        ops.linear_xf(xf, M, w, "f32", out=o, splitk=2)
    else:
        ops.linear(x, w, "f32", out=o, splitk=2)
torch.cuda.synchronize()
ref = x.float() @ ops.unshuffle_weight(w.data, N, K).float().t()
print(mode, M, "max err", (o.sum(0) - ref).abs().max().item(), flush=True)

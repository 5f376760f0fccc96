"""Run one prefill GEMM back to back (for rocprofv3 --pmc passes): shape M N K epi cfg [iters] [--cold] [--vendor].
cfg: stream-K configuration code (ops.SK_CFGS index, + 8 whole tiles, + 16 + 32 * epilogue mode; -2 = the engine's
table).  --cold: a 512 MiB cache-flushing write before every call (the engine's case: weights from HBM).  --vendor: the
same product on hipBLASLt (torch.mm / addmm) instead.  Random operands.  Example: probe_gemm_sk.py 2048 3072 8192 res -2 30 --cold"""
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

argv = [a for a in sys.argv[1:] if not a.startswith("--")]
cold, vendor = "--cold" in sys.argv, "--vendor" in sys.argv
M, N, K, epi, cfg = int(argv[0]), int(argv[1]), int(argv[2]), argv[3], int(argv[4])
it = int(argv[5]) if len(argv) > 5 else 50
dev = torch.device("cuda:0")
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
pw = ops.PackedWeight.from_dense(w)
wt = w.t()
out = torch.zeros(M, N // 2 if epi == "silu" else N, device=dev,
                  dtype=torch.float32 if epi in ("f32", "res") else torch.bfloat16)
y16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
flush = torch.empty(128 << 20, device=dev) if cold else None


def call():
    if not vendor:
        ops.gemm_sk(x, pw.data, N, out, epi, cfg=None if cfg == -2 else cfg)
    elif epi == "res":
        torch.addmm(out, x, wt, out_dtype=torch.float32, out=out)
    elif epi == "silu":
        torch.mm(x, wt, out=y16)
    else:
        torch.mm(x, wt, out=out)


for _ in range(3):
    call()
torch.cuda.synchronize()
ts = []
for _ in range(it):
    if cold:
        flush.fill_(1.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1000)
us = sorted(ts)[len(ts) // 2]
print(f"{M}x{N}x{K} {epi} cfg {cfg} {'vendor' if vendor else 'hand'} {'cold' if cold else 'warm'}: {us:.1f} us, "
      f"{2.0 * M * N * K / us / 1e6:.0f} TF")

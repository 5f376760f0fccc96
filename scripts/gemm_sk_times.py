"""Stream-K prefill GEMM times of the loaded build (cross-build A/Bs: run in turns under LSA_HIP_SO=variants/<x>.so and
without): each shape at the engine's table configuration, warm and cold (512 MiB write before each call), median of
7.  One JSON line.  Usage: gemm_sk_times.py [tag] [xf]: xf = also the fragment-major operands (ops.to_xfrag X, and
the SiLU output in that layout), interleaved with the row-major calls in the same process (keys ..._xf)."""
import json
import statistics as st
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

SHAPES = {"3b_o_m2048": (2048, 3072, 3072, "res"), "3b_down_m2048": (2048, 3072, 8192, "res"),
          "3b_qkv_m2048": (2048, 5120, 3072, "bf16"), "3b_gateup_m2048": (2048, 16384, 3072, "silu"),
          "7b_qkv_m300": (300, 12288, 4096, "bf16"), "7b_o_m300": (300, 4096, 4096, "res"),
          "7b_down_m300": (300, 4096, 11008, "res"), "3b_o_m512": (512, 3072, 3072, "res"),
          "7b_qkv_m1024": (1024, 12288, 4096, "bf16"), "7b_down_m4096": (4096, 4096, 11008, "res")}
dev = torch.device("cuda:0")
flush = torch.empty(128 << 20, device=dev)
out_rec = {"tag": sys.argv[1] if len(sys.argv) > 1 else "", "build": ops.ext().__file__}
XF = len(sys.argv) > 2 and sys.argv[2] == "xf"
for name, (M, N, K, epi) in SHAPES.items():
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16).to(dev)
    pw = ops.PackedWeight.from_dense(w)
    out = torch.zeros(M, N // 2 if epi == "silu" else N, device=dev,
                      dtype=torch.float32 if epi in ("f32", "res") else torch.bfloat16)
    xf = ops.to_xfrag(x)
    outf = torch.zeros(ops.xfrag_tiles(M) * 16 * (N // 2), device=dev, dtype=torch.bfloat16) if epi == "silu" else out
    arms = {"": lambda: ops.gemm_sk(x, pw.data, N, out, epi)}
    if XF:
        arms["_xf"] = lambda: ops.gemm_sk(xf, pw.data, N, outf, epi, rows=M, xf_out=epi == "silu")
    for mode in ("warm", "cold"):
        ts = {a: [] for a in arms}
        for _ in range(8):
            for a, fn in arms.items():
                if mode == "cold":
                    flush.fill_(1.0)
                else:
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts[a].append(e0.elapsed_time(e1) * 1000)
        for a in arms:
            out_rec[f"{name}_{mode}{a}"] = round(st.median(ts[a][1:]), 2)
print(json.dumps(out_rec), flush=True)

"""W8A8 fp8 prefill GEMM (block-scaled 16x16x128 f8f6f4 MFMA, kernels/gemm_fp8_tile.hip) vs the bf16 256^2
tile kernel and vs the weight-only fp8 path it replaces (dequantise the layer to bf16 + bf16 tile GEMM), at
the BASELINE prefill shapes.  Times the GEMM alone and with the per-token activation quantisation; random
operands; relative error vs the fp32 product of the bf16 activations and the dequantised weights.
One JSON line per shape.

    python scripts/bench_fp8_prefill.py [shape,...]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
EPI = {"bf16": 0, "f32": 1, "silu": 2}


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    reps = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        reps.append(e0.elapsed_time(e1) * 1000 / it)
    return sorted(reps)[1]


shapes = {"7b_qkv": (4096, 12288, 4096, "bf16"), "7b_o": (4096, 4096, 4096, "f32"),
          "7b_gateup": (4096, 22016, 4096, "silu"), "7b_down": (4096, 4096, 11008, "f32"),
          "3b_qkv": (2048, 5120, 3072, "bf16"), "3b_gateup": (2048, 16384, 3072, "silu"),
          "3b_down": (2048, 3072, 8192, "f32"), "7b_qkv_m512": (512, 12288, 4096, "bf16"),
          "sq8192": (8192, 8192, 8192, "bf16")}
if len(sys.argv) > 1:
    shapes = {k: v for k, v in shapes.items() if k in sys.argv[1].split(",")}
e = ops.ext()
for name, (M, N, K, epi) in shapes.items():
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    pw8 = ops.PackedWeight.from_dense(w, "fp8")
    pwb = ops.PackedWeight.from_dense(w)
    wd = pw8.dense().float()
    ncol = N // 2 if epi == "silu" else N
    out = torch.empty(M, ncol, device=dev, dtype=torch.float32 if epi == "f32" else torch.bfloat16)
    ref = x.float() @ wd.t()
    if epi == "silu":
        r3 = ref.view(M, N // 32, 2, 16)
        ref = (torch.nn.functional.silu(r3[:, :, 0]) * r3[:, :, 1]).reshape(M, N // 2)
    flops = 2.0 * M * N * K
    x8, sx = ops.quantize_rows_fp8(x)
    dq = torch.empty(N * K, device=dev, dtype=torch.bfloat16)
    res = {"shape": name, "M": M, "N": N, "K": K, "epi": epi}
    arms = (("fp8_w8a8_gemm", lambda: e.fp8_gemm_t256(x8, sx, pw8.data, pw8.scale, N, out, EPI[epi], 1)),
            ("fp8_w8a8_with_quant", lambda: (ops.quantize_rows_fp8(x),
                                             e.fp8_gemm_t256(x8, sx, pw8.data, pw8.scale, N, out, EPI[epi], 1))),
            ("fp8_weight_only_dequant", lambda: (e.fp8_dequant(pw8.data, pw8.scale, N, K, dq),
                                                 ops.gemm_sk(x, dq, N, out, epi))),
            ("bf16_stream_k", lambda: ops.gemm_sk(x, pwb.data, N, out, epi)))
    for kname, fn in arms:
        fn()
        torch.cuda.synchronize()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        us = timeit(fn)
        res[kname] = {"us": round(us, 1), "TF": round(flops / us / 1e6, 1), "rel_err": float(f"{err:.2e}")}
    print(json.dumps(res), flush=True)
    del pw8, pwb, dq, wd
    torch.cuda.empty_cache()

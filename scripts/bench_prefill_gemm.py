"""Prefill GEMM on MI355X: 128^2 tile kernel vs 256^2 tile kernel vs hipBLASLt (torch.matmul) at the
prefill shapes of the BASELINE configs (7B: 32 x 128-token prompts = 4096 rows; 3B: one 2k prompt),
plus a square 8192^3 reference.  Random operands (TF/s on zero-filled data reads high).  Checks each
kernel against an fp32 product first."""
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
          "3b_down": (2048, 3072, 8192, "f32"), "7b_qkv_m300": (300, 12288, 4096, "bf16"),
          "7b_gateup_m300": (300, 22016, 4096, "silu"), "7b_gateup_m1024": (1024, 22016, 4096, "silu"),
          "3b_gateup_m300": (300, 16384, 3072, "silu"),
          "sq8192": (8192, 8192, 8192, "bf16")}
if len(sys.argv) > 1:
    shapes = {k: v for k, v in shapes.items() if k in sys.argv[1].split(",")}
e = ops.ext()
for name, (M, N, K, epi) in shapes.items():
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    pw = ops.PackedWeight.from_dense(w)
    ncol = N // 2 if epi == "silu" else N
    out = torch.empty(M, ncol, device=dev, dtype=torch.float32 if epi == "f32" else torch.bfloat16)
    ref = x.float() @ w.float().t()
    if epi == "silu":
        r3 = ref.view(M, N // 32, 2, 16)
        ref = (torch.nn.functional.silu(r3[:, :, 0]) * r3[:, :, 1]).reshape(M, N // 2)
    res = {"shape": name, "M": M, "N": N, "K": K, "epi": epi}
    flops = 2.0 * M * N * K
    mtt = (M + 255) // 256 * 16  # fragment-major X over whole 256-row tiles
    xp = torch.zeros(mtt * 16, K, device=dev, dtype=torch.bfloat16)
    xp[:M] = x
    xf = xp.view(mtt, 16, K // 32, 4, 8).permute(2, 0, 3, 1, 4).contiguous().view(-1)
    for kname, fn in (("tile128", lambda: e.gemm(x, pw.data, N, out, EPI[epi], 1, 1, 4, 4, 0)),
                      ("tile256", lambda: e.gemm_t256(x, pw.data, N, out, EPI[epi])),
                      ("tile256_xf", lambda: e.gemm_t256_xf(xf, mtt, M, pw.data, N, out, EPI[epi]))):
        fn()
        torch.cuda.synchronize()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        us = timeit(fn)
        res[kname] = {"us": round(us, 1), "TF": round(flops / us / 1e6, 1), "rel_err": float(f"{err:.2e}")}
    wt = w.t()
    us = timeit(lambda: torch.matmul(x, wt))
    res["hipblaslt"] = {"us": round(us, 1), "TF": round(flops / us / 1e6, 1)}
    o32 = torch.empty(M, N, device=dev, dtype=torch.float32)
    us = timeit(lambda: torch.mm(x, wt, out_dtype=torch.float32, out=o32))
    res["hipblaslt_f32out"] = {"us": round(us, 1), "TF": round(flops / us / 1e6, 1)}
    if epi == "silu":  # vendor GEMM (f32 out, gate/up rows interleaved per 16 as packed) + the SiLU*up pass
        def blas_silu():
            torch.mm(x, wt, out_dtype=torch.float32, out=o32)
            e.silu_parts(o32.view(1, M, N), out)
        blas_silu()
        torch.cuda.synchronize()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        us = timeit(blas_silu)
        res["hipblaslt_silu"] = {"us": round(us, 1), "TF": round(flops / us / 1e6, 1), "rel_err": float(f"{err:.2e}")}
    print(json.dumps(res), flush=True)
    del x, w, pw, out, ref
    torch.cuda.empty_cache()

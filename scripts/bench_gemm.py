"""Decode-GEMM sweep on the GPU: effective HBM bandwidth of ops.linear for the 7B / 3B decode
shapes at M = 1 and 32 over (nb, splitk).  Weights rotate over enough copies (> 256 MiB) that every
call streams from HBM, as in a real decode step (13.5 GB of weights per token)."""
import sys, time, json
import torch
sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops

dev = torch.device("cuda:0")
SHAPES = {  # name: (N, K, epi)
    "7b_qkv": (12288, 4096, "f32"), "7b_o": (4096, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"),
    "7b_down": (4096, 11008, "f32"), "7b_head": (32000, 4096, "f32"), "7b_gateup_f32": (22016, 4096, "f32"),
    "3b_qkv": (5120, 3072, "f32"), "3b_o": (3072, 3072, "f32"), "3b_gateup": (16384, 3072, "silu"),
    "3b_down": (3072, 8192, "f32"), "3b_head": (128256, 3072, "f32"), "3b_gateup_f32": (16384, 3072, "f32"),
}
Ms = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 32]
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
if only:
    SHAPES = {k: v for k, v in SHAPES.items() if k in only}
res = []
for name, (N, K, epi) in SHAPES.items():
    nbytes = N * K * 2
    ncopy = max(2, (600 << 20) // nbytes + 1)
    ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(ncopy)]
    for M in Ms:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        best = None
        for waves, xl, dv in ((4, 0, 1), (4, 0, 2), (8, 0, 2), (4, 0, 4), (8, 0, 4)):
         for nb in (1, 2, 4):
            if (N // 16) % nb or (epi == "silu" and nb == 1) or (M > 32 and nb > 2):
                continue
            for sk in ((1, 2, 4, 8) if epi == "f32" else (1,)):
                if K // 32 // sk < 8:
                    continue
                out = torch.empty(sk * M * N if epi == "f32" else M * N, device=dev,
                                  dtype=torch.float32 if epi == "f32" else torch.bfloat16)
                o = out.view(sk, M, N) if epi == "f32" else out.view(M, N)[:, : N // 2 if epi == "silu" else N]
                if epi == "silu":
                    o = out[: M * N // 2].view(M, N // 2)
                for i in range(3):
                    ops.linear(x, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb, waves=waves, div=dv)
                torch.cuda.synchronize()
                it = 40
                reps = []
                for _rep in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(it):
                        ops.linear(x, ws[i % ncopy], epi, out=o, splitk=sk, nb=nb, waves=waves, div=dv)
                    e1.record(); torch.cuda.synchronize()
                    reps.append(e0.elapsed_time(e1) * 1000 / it)
                us = sorted(reps)[1]
                tbs = nbytes / us / 1e6
                r = dict(shape=name, M=M, waves=waves, xlds=xl, div=dv, nb=nb, splitk=sk, us=round(us, 2), TBps=round(tbs, 3))
                res.append(r)
                if best is None or us < best["us"]:
                    best = r
        print("BEST", json.dumps(best), flush=True)
    del ws
    torch.cuda.empty_cache()
json.dump(res, open("gpurun_out/gemm_sweep.json", "w"), indent=0)
# tuning table: (N, K, epi, M-class) -> best (waves, nb, splitk)
table = {}
for r in res:
    N, K, epi = SHAPES[r["shape"]]
    key = f"{N}x{K}:{epi}:{'s' if r['M'] <= 16 else 'm'}"
    if key not in table or r["us"] < table[key]["us"]:
        table[key] = {"waves": r["waves"], "div": r["div"], "nb": r["nb"], "splitk": r["splitk"], "us": r["us"], "TBps": r["TBps"]}
json.dump(table, open("gpurun_out/gemm_tuning.json", "w"), indent=1)

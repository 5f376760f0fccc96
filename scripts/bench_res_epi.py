"""Norm-folded decode A/B per row-parallel projection (o / down): the split-K f32-slab GEMM followed by the
add_rmsnorm launch (the unfused path) vs one GEMM with the residual epilogue (h += y, x = bf16(h), row
sums of squares; no norm launch), swept over (nb, waves, div).  Also times the column-parallel GEMMs
(qkv f32 slabs, gate_up SiLU) with and without the rownorm row scale.  Weights rotate over > 600 MiB so
they stream from HBM; us per call (median of 3 x 30).  One JSON line per (shape, M, kind).

    python scripts/bench_res_epi.py [Ms] [bf16|fp8] [--rowp-only]

Each row-parallel line carries a ready "tune" entry (key "NxK:res:b<M>[:fp8]") when the sweep's best beats
the f32 pick by > 3 %; scripts/merge_tuning.py folds them into ops/gemm_tuning.json.
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ROWP = {"7b_o": (4096, 4096), "7b_down": (4096, 11008), "3b_o": (3072, 3072), "3b_down": (3072, 8192)}
COLP = {"7b_qkv": (12288, 4096, "f32"), "7b_gateup": (22016, 4096, "silu"), "3b_qkv": (5120, 3072, "f32"),
        "3b_gateup": (16384, 3072, "silu")}
_pos = [a for a in sys.argv[1:] if not a.startswith("--")]
Ms = [int(a) for a in _pos[0].split(",")] if _pos else [1, 8, 32]
KIND = _pos[1] if len(_pos) > 1 else "bf16"


def timeit(fn, it=30):
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


def weights(N, K):
    nbytes = N * K * (1 if KIND == "fp8" else 2)
    ncopy = max(2, (600 << 20) // nbytes + 1)
    return [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), KIND)
            for _ in range(ncopy)], ncopy


for name, (N, K) in ROWP.items():
    ws, ncopy = weights(N, K)
    for M in Ms:
        xf = 16 < M <= 64
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        af = ops.to_xfrag(a) if xf else a
        h = torch.randn(M, N, device=dev)
        xout = torch.zeros(ops.xfrag_tiles(M) * 16 * N if xf else M * N, device=dev, dtype=torch.bfloat16)
        ss = torch.zeros(M, device=dev, dtype=torch.int64)
        g = torch.ones(N, device=dev, dtype=torch.bfloat16)

        def lin(x, w, epi, **kw):
            return ops.linear_xf(x, M, w, epi, **kw) if xf else ops.linear(x, w, epi, **kw)

        nb0, sk0, wv0, dv0 = ops.pick_gemm_config(M, N, K, "f32", xf=xf, kind=KIND)
        parts = torch.empty(sk0, M, N, device=dev)

        def old(i):
            lin(af, ws[i % ncopy], "f32", out=parts, splitk=sk0)
            ops.add_rmsnorm(h, g, 1e-5, xout if xf else xout.view(M, N), parts=parts, rows=M, xf=xf)

        tk = torch.zeros(N // 16, device=dev, dtype=torch.int32)
        xo = xout if xf else xout.view(M, N)
        res = {"shape": name, "M": M, "kind": KIND, "xf": xf, "old_cfg": [nb0, sk0, wv0, dv0],
               "old_gemm_plus_norm_us": round(timeit(old), 2),
               "res_same_cfg_us": round(timeit(lambda i: lin(af, ws[i % ncopy], "res", out=parts, splitk=sk0,
                                                             res=(h, xo, ss, tk))), 2)}
        best = None
        for nb in (1, 2, 4, 6, 8):
            if (M > 32 and nb > 2) or (N // 16) % nb or (nb == 6 and not 16 < M <= 32):
                continue
            for sk in (1, 2, 4, 8):
                if K // 32 // sk < 8:
                    continue
                pb = torch.empty(sk, M, N, device=dev)
                for waves, dv in (((4, 1), (4, 2), (4, 4), (8, 2)) if KIND == "bf16" else ((4, 4),)):
                    if nb >= 6 and (KIND != "bf16" or (waves, dv) not in ((4, 1), (4, 2))):
                        continue
                    if waves == 16 and (M > 16 or nb > 2):  # the 16-wave kernel: one row tile, nb <= 2
                        continue
                    us = timeit(lambda i: lin(af, ws[i % ncopy], "res", out=pb, splitk=sk, res=(h, xo, ss, tk),
                                              nb=nb, waves=waves, div=dv))
                    if best is None or us < best[1]:
                        best = ((nb, sk, waves, dv), us)
        res["res_best"] = list(best[0])
        res["res_best_us"] = round(best[1], 2)
        if best[1] < 0.97 * res["res_same_cfg_us"] and M in (1, 2, 4, 8, 16, 32, 64):
            nb, sk, wv, dv = best[0]
            res["tune"] = {f"{N}x{K}:res:b{M}" + (":fp8" if KIND == "fp8" else ""):
                           {"nb": nb, "splitk": sk, "waves": wv, "div": dv, "us": round(best[1], 2),
                            "note": f"scripts/bench_res_epi.py: f32 pick {res['res_same_cfg_us']} us"}}
        print(json.dumps(res), flush=True)
    del ws
    torch.cuda.empty_cache()

for name, (N, K, epi) in ({} if "--rowp-only" in sys.argv else COLP).items():
    ws, ncopy = weights(N, K)
    for M in Ms:
        xf = 16 < M <= 64
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xin = ops.to_xfrag(x) if xf else x
        ss = ops.ss_q24(x.float().pow(2).sum(1))
        nb, sk, wv, dv = ops.pick_gemm_config(M, N, K, epi, xf=xf, kind=KIND)
        o = torch.empty(sk, M, N, device=dev) if epi == "f32" else torch.empty(
            ops.xfrag_tiles(M) * 16 * (N // 2) if xf else M * N // 2, device=dev, dtype=torch.bfloat16)
        oo = o if (epi == "f32" or xf) else o.view(M, N // 2)

        def run(rn):
            if xf:
                return lambda i: ops.linear_xf(xin, M, ws[i % ncopy], epi, out=oo, splitk=sk, rownorm=rn)
            return lambda i: ops.linear(xin, ws[i % ncopy], epi, out=oo, splitk=sk, rownorm=rn)

        print(json.dumps({"shape": name, "M": M, "kind": KIND, "cfg": [nb, sk, wv, dv],
                          "plain_us": round(timeit(run(None)), 2),
                          "rownorm_us": round(timeit(run((ss, 1e-5))), 2)}), flush=True)
    del ws
    torch.cuda.empty_cache()

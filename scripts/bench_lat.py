"""Latency-path GEMV sweep (csrc/kernels/decode_lat.hip) at batch 1 on the 7B / 3B decode shapes.

Each config runs over R weight copies totalling > 512 MB in a row (a back-to-back replay of ONE copy would stream from
the 256 MB Infinity Cache, not HBM), timed with hipEvents; one JSON line per (shape, config): median us per call and
the weight stream rate.  ``python scripts/bench_lat.py [--M 1] [--proj qkv,o,gate_up,down]``
"""
import argparse
import itertools
import json
import math
import statistics
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

SHAPES = {  # model: (d, H, Hkv, ffn, ctx)
    "7b": (4096, 32, 32, 11008, 200),
    "3b": (3072, 24, 8, 8192, 2100),
}


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        n = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / n)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=1)
    ap.add_argument("--proj", default="qkv,o,gate_up,down")
    ap.add_argument("--models", default="7b,3b")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    M = args.M
    for model in args.models.split(","):
        d, H, Hkv, ffn, ctx = SHAPES[model]
        shapes = {"qkv": ((H + 2 * Hkv) * 128, d), "o": (d, H * 128), "gate_up": (2 * ffn, d), "down": (d, ffn)}
        for proj in args.proj.split(","):
            N, K = shapes[proj]
            R = max(2, math.ceil(512e6 / (N * K * 2)))
            ws = [ops.PackedWeight.from_dense((torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16))
                  for _ in range(R)]
            hq = ops.to_q32(torch.randn(M, d if proj != "down" else d, device=dev))
            hq_in = ops.to_q32(torch.randn(M, K, device=dev))
            ss = torch.zeros(64, dtype=torch.int64, device=dev)
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            out = torch.empty(8 * M * N, device=dev)
            act = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
            nsplit = (ctx + 63) // 64
            opart = torch.randn(M, H, nsplit, 128, device=dev)
            ml = torch.stack([torch.randn(M, H, nsplit, device=dev), torch.rand(M, H, nsplit, device=dev) + 1], -1)
            pos = torch.full((M,), ctx - 1, dtype=torch.int32, device=dev)
            nbt = N // 16
            if proj == "o":
                cands = [(nb, H, wv) for nb in (2, 4, 8) for wv in (4, 8) if nbt % nb == 0]
                cands += [(nb, H // 2, wv) for nb in (2, 4) for wv in (4, 8) if nbt % nb == 0]
            elif proj == "gate_up":
                cands = [(nb, 1, wv) for nb in (2, 4, 8) for wv in (4, 8) if nbt % nb == 0]
            else:
                cands = [(nb, sk, wv) for nb, sk, wv in itertools.product((1, 2, 4, 8), (1, 2, 4, 8), (4, 8))
                         if nbt % nb == 0 and (nbt // nb) * sk >= 96 and (nbt // nb) * sk <= 4096]
            for nb, sk, wv in cands:
                def run():
                    for w in ws:
                        ss.zero_()
                        if proj in ("qkv",):
                            ops.lat_linear(w, M, "hq", "f32", sk, nb, wv, hq=hq_in, ss=ss, out=out)
                        elif proj == "gate_up":
                            ops.lat_linear(w, M, "hq", "silu", sk, nb, wv, hq=hq_in, ss=ss, act=act)
                        elif proj == "o":
                            ops.lat_linear(w, M, "part", "atom", sk, nb, wv, part=(opart, ml, pos, (1, nsplit, 0), H),
                                           hq_out=hq)
                        else:
                            ops.lat_linear(w, M, "act", "atom", sk, nb, wv, x=x, hq_out=hq)
                    return len(ws)
                try:
                    run()
                    torch.cuda.synchronize()
                    us = timed(run)
                except RuntimeError as e:  # an invalid combination (LDS, split) is reported, not fatal
                    print(json.dumps({"model": model, "proj": proj, "nb": nb, "sk": sk, "waves": wv, "error": str(e)[:80]}))
                    continue
                # the ss.zero_() per call is part of the time: subtract a memset's ~2 us? keep it honest: report raw
                print(json.dumps({"model": model, "proj": proj, "N": N, "K": K, "M": M, "nb": nb, "sk": sk, "waves": wv,
                                  "us": round(us, 2), "TBps": round(N * K * 2 / us / 1e6, 2)}), flush=True)
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

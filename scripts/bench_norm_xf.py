"""Prefill RMSNorm (h alone -> bf16) times: row-major, fragment-major from the row-per-workgroup kernel, and
fragment-major from the 16-row-tile kernel (ext.rmsnorm_xf_tile_min picks which writes the layout), interleaved,
median of 20 (us).  One JSON line per shape."""
import json
import statistics as st
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for D in (3072, 4096):
    for M in (300, 512, 1024, 2048, 4096):
        h = torch.randn(M, D, device=dev)
        w = torch.randn(D, device=dev).to(torch.bfloat16)
        xr = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
        xf = torch.empty(ops.xfrag_tiles(M) * 16 * D, device=dev, dtype=torch.bfloat16)
        tile = ops.ext().rmsnorm_xf_tile_min
        arms = {"row": (lambda: None, lambda: ops.add_rmsnorm(h, w, 1e-5, xr, write_h=False)),
                "xf_rowwg": (lambda: tile(1 << 30), lambda: ops.add_rmsnorm(h, w, 1e-5, xf, write_h=False, rows=M, xf=True)),
                "xf_tile": (lambda: tile(65), lambda: ops.add_rmsnorm(h, w, 1e-5, xf, write_h=False, rows=M, xf=True))}
        ts = {a: [] for a in arms}
        for _ in range(21):
            for a, (setup, fn) in arms.items():
                setup()
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts[a].append(e0.elapsed_time(e1) * 1000)
        tile(1024)
        print(json.dumps({"M": M, "D": D, **{a: round(st.median(v[1:]), 2) for a, v in ts.items()}}), flush=True)

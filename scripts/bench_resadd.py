"""Residual-add launch cost on MI355X: ops.res_add_ss (one wave per 512 columns, Q24 atomics) vs add_rmsnorm (one
workgroup per row) at the decode shapes, each timed as 200 back-to-back launches inside one captured hipGraph (the
decode step's setting: dependent launches, no host gaps), us per launch, median of 3.  With LSA_HIP_SO pointing at an
experiment build (scripts/build_variants.sh) the same numbers for that variant."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
tag = sys.argv[1] if len(sys.argv) > 1 else "default"
for (B, d, S) in ((32, 4096, 4), (32, 4096, 2), (1, 3072, 4), (1, 4096, 2)):
    xf = 16 < B <= 64
    h = torch.randn(64, d, device=dev)
    parts = torch.randn(S, B, d, device=dev)
    xn = torch.zeros(ops.xfrag_tiles(B) * 16 * d if xf else B * d, device=dev, dtype=torch.bfloat16)
    ss = torch.zeros(64, device=dev, dtype=torch.int64)
    g = torch.ones(d, device=dev, dtype=torch.bfloat16)
    xo = xn if xf else xn.view(B, d)
    res = {"tag": tag, "B": B, "d": d, "slabs": S}
    for name, fn in (("res_add_ss", lambda: ops.res_add_ss(h[:B], parts, xo, B, ss, xf=xf)),
                     ("add_rmsnorm", lambda: ops.add_rmsnorm(h[:B], g, 1e-5, xo, parts=parts, rows=B, xf=xf))):
        fn()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(gr, stream=s):
                for _ in range(200):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        gr.replay()
        torch.cuda.synchronize()
        reps = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            reps.append(e0.elapsed_time(e1) * 1000 / 200)
        res[name + "_us"] = round(sorted(reps)[1], 3)
    print(json.dumps(res), flush=True)

"""Stream-K tile configurations re-timed with fragment-major operands (the engine's prefill layout since round 6):
every configuration (+ 8: whole tiles) on the given prefill shapes, cold (512 MiB write before each call) median of
7, against the table's pick.  One JSON line per shape.  Usage: sweep_sk_xf.py [shape,...]"""
import json
import statistics as st
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

SHAPES = {"3b_qkv_m2048": (2048, 5120, 3072, "bf16"), "3b_o_m2048": (2048, 3072, 3072, "res"),
          "3b_gateup_m2048": (2048, 16384, 3072, "silu"), "3b_down_m2048": (2048, 3072, 8192, "res"),
          "7b_qkv_m4096": (4096, 12288, 4096, "bf16"), "7b_gateup_m4096": (4096, 22016, 4096, "silu"),
          "7b_down_m4096": (4096, 4096, 11008, "res"), "7b_o_m4096": (4096, 4096, 4096, "res"),
          "7b_qkv_m300": (300, 12288, 4096, "bf16"), "7b_o_m300": (300, 4096, 4096, "res"),
          "7b_gateup_m300": (300, 22016, 4096, "silu"), "7b_down_m300": (300, 4096, 11008, "res")}
names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(SHAPES)
dev = torch.device("cuda:0")
flush = torch.empty(128 << 20, device=dev)
for name in names:
    M, N, K, epi = SHAPES[name]
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16).to(dev)
    pw = ops.PackedWeight.from_dense(w)
    xf = ops.to_xfrag(x)
    out = (torch.zeros(ops.xfrag_tiles(M) * 16 * (N // 2), device=dev, dtype=torch.bfloat16) if epi == "silu" else
           torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == "res" else torch.bfloat16))
    table = ops.sk_config(M, N, K, epi)
    rec = {"shape": name, "table_cfg": table}
    for cfg in list(range(8)) + list(range(8, 16)):
        if epi == "silu" and not ops.sk_cfg_pairs(cfg):
            continue
        ts = []
        for _ in range(8):
            flush.fill_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.gemm_sk(xf, pw.data, N, out, epi, cfg=cfg, rows=M, xf_out=epi == "silu")
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000)
        rec[ops.sk_cfg_tag(cfg)] = round(st.median(ts[1:]), 2)
    print(json.dumps(rec), flush=True)

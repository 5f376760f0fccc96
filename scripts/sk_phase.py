"""Where a one-phase K-tile of the stream-K prefill GEMM spends its cycles (128-row tiles, NBUF 4): per wave, s_memtime
cycles of [fragment reads + LDS-DMA issue + counted waits], [barrier 1], [MFMA issue], [barrier 2], divided by its
K-tiles; medians over waves, split by wave group (wm 0 / 1: the ping-pong halves), warm and cold.  Needs the
LSA_SK_PHASE build: python scripts/build_variant.py phase gemm_tile256.hip -DLSA_SK_PHASE, then run under
LSA_HIP_SO=variants/phase.so.  Usage: sk_phase.py [shape,...] [cfg]"""
import json
import statistics as st
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

SHAPES = {"3b_o_m2048": (2048, 3072, 3072, "res", 60), "3b_down_m2048": (2048, 3072, 8192, "res", 60),
          "7b_qkv_m300": (300, 12288, 4096, "bf16", None), "7b_o_m1024": (1024, 4096, 4096, "res", None),
          "3b_o_m2048_t3": (2048, 3072, 3072, "res", 16 + 32 + 8 + 3)}
names = sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1] else list(SHAPES)
dev = torch.device("cuda:0")
stamps = torch.zeros(256 * 8, 8, dtype=torch.int64, device=dev)
flush = torch.empty(128 << 20, device=dev)
ext = ops.ext()
for name in names:
    M, N, K, epi, cfg = SHAPES[name]
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16).to(dev)
    pw = ops.PackedWeight.from_dense(w)
    out = torch.zeros(M, N // 2 if epi == "silu" else N, device=dev,
                      dtype=torch.float32 if epi in ("f32", "res") else torch.bfloat16)
    for mode in ("warm", "cold"):
        per = {0: [], 1: []}
        for it in range(4):
            if mode == "cold":
                flush.fill_(1.0)
            else:
                ops.gemm_sk(x, pw.data, N, out, epi, cfg=cfg)
            torch.cuda.synchronize()
            stamps.zero_()
            ext.sk_set_stamps(stamps)
            ops.gemm_sk(x, pw.data, N, out, epi, cfg=cfg)
            torch.cuda.synchronize()
            ext.sk_set_stamps(None)
            s = stamps.view(256, 8, 8).cpu()
            for b in range(256):
                for wv in range(8):
                    kt = int(s[b, wv, 4])
                    if kt > 0:
                        per[wv // 4].append([int(s[b, wv, k]) / kt for k in range(7)])
        rec = {"shape": name, "M": M, "N": N, "K": K, "epi": epi, "cfg": cfg, "table_cfg": ops.sk_config(M, N, K, epi),
               "mode": mode}
        for grp, rows in per.items():
            if rows:
                med = [round(st.median(r[k] for r in rows)) for k in range(7)]
                rec[f"wm{grp}"] = {"reads_dma_waits": med[0], "of_which_reads": med[5], "of_which_dma_issue": med[6],
                                   "barrier1": med[1], "mfma": med[2], "barrier2": med[3], "total": sum(med[:4]),
                                   "waves": len(rows)}
        print(json.dumps(rec), flush=True)

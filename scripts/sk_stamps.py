"""Where a stream-K prefill GEMM's time goes (csrc/kernels/gemm_tile256.hip g_sk_stamps): per workgroup, launch
skew (entry - first entry), pipeline fill (first segment's prologue), K loop (per K-tile), epilogue + stream-K fixup
(last loop end -> exit), and the kernel span (first entry -> last exit) next to the HIP-event time, warm and cold
(a 512 MiB cache-flushing write before the call: the engine's case, weights from HBM).  The effective shader clock
comes from s_memtime over the K loop.  Needs the stamped build: LSA_HIP_EXTRA=-DLSA_SK_STAMPS (ops/build.py).
Usage: sk_stamps.py [shape,...] [cfg]   (shapes: bench_prefill_gemm names)"""
import json
import statistics as st
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

SHAPES = {"3b_qkv_m2048": (2048, 5120, 3072, "bf16"), "3b_o_m2048": (2048, 3072, 3072, "res"),
          "3b_gateup_m2048": (2048, 16384, 3072, "silu"), "3b_down_m2048": (2048, 3072, 8192, "res"),
          "7b_qkv_m128": (128, 12288, 4096, "bf16"), "7b_gateup_m128": (128, 22016, 4096, "silu"),
          "7b_qkv_m4096": (4096, 12288, 4096, "bf16")}
names = sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1] else list(SHAPES)
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else None
dev = torch.device("cuda:0")
stamps = torch.zeros(2048, 8, dtype=torch.int64, device=dev)
flush = torch.empty(128 << 20, device=dev)
ext = ops.ext()


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


for name in names:
    M, N, K, epi = SHAPES[name]
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16).to(dev)
    pw = ops.PackedWeight.from_dense(w)
    out = torch.zeros(M, N // 2 if epi == "silu" else N, device=dev,
                      dtype=torch.float32 if epi in ("f32", "res") else torch.bfloat16)
    for mode in ("warm", "cold"):
        recs = []
        for it in range(6):
            if mode == "cold":
                flush.fill_(1.0)
            else:
                ops.gemm_sk(x, pw.data, N, out, epi, cfg=cfg)
            torch.cuda.synchronize()
            stamps.zero_()
            ext.sk_set_stamps(stamps)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.gemm_sk(x, pw.data, N, out, epi, cfg=cfg)
            e1.record()
            torch.cuda.synchronize()
            ext.sk_set_stamps(None)
            s = stamps.cpu()
            live = s[:, 3] > 0
            s = s[live]
            t0 = int(s[:, 0].min())
            ent = [(int(a) - t0) * 10 / 1000 for a in s[:, 0]]  # us (100 MHz ticks)
            fill = [(int(b) - int(a)) * 10 / 1000 for a, b in zip(s[:, 0], s[:, 1])]
            loop = [(int(c) - int(b)) * 10 / 1000 for b, c in zip(s[:, 1], s[:, 2])]
            epi_t = [(int(d) - int(c)) * 10 / 1000 for c, d in zip(s[:, 2], s[:, 3])]
            ext_ = [(int(d) - t0) * 10 / 1000 for d in s[:, 3]]
            kts = [int(k) for k in s[:, 4]]
            per_kt = [lp / max(1, k) for lp, k in zip(loop, kts)]
            clk = [(int(b7) - int(b6)) / max(1e-9, (int(c) - int(b)) * 10) for b6, b7, b, c in
                   zip(s[:, 6], s[:, 7], s[:, 1], s[:, 2]) if int(c) > int(b)]
            recs.append({"event_us": e0.elapsed_time(e1) * 1000, "span_us": max(ext_), "wgs": int(live.sum()),
                         "entry_skew_p50": pct(ent, .5), "entry_skew_max": max(ent),
                         "fill_p50": pct(fill, .5), "fill_max": max(fill),
                         "loop_p50": pct(loop, .5), "loop_max": max(loop), "kt_per_wg": st.median(kts),
                         "us_per_ktile_p50": pct(per_kt, .5),
                         "epi_p50": pct(epi_t, .5), "epi_max": max(epi_t),
                         "exit_p10": pct(ext_, .1), "exit_p50": pct(ext_, .5), "exit_max": max(ext_),
                         "segs_max": int(s[:, 5].max()), "ghz_p50": pct(clk, .5) if clk else None})
        med = {k: round(st.median(r[k] for r in recs[1:]), 2) if isinstance(recs[1][k], (int, float)) else recs[1][k]
               for k in recs[1]}
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "epi": epi, "cfg": cfg, "mode": mode, **med}),
              flush=True)

"""A/B of the stream-K prefill GEMM's K-loop schedules on the 128-row tiles: four phases per K-tile with three buffers
(default) vs one phase with four buffers (ext.gemm_sk_one_phase), per shape at the engine's tile choice and at forced
128-row configurations; warm and cold (512 MiB cache flush before each call: the engine's weights-from-HBM case).
Arms interleaved in one process (cdna_hip_programming.md §5.4 rule 24), median of the rounds.
Usage: ab_sk_sched.py [shape,...]"""
import json
import statistics as st
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

SHAPES = {"3b_qkv_m2048": (2048, 5120, 3072, "bf16"), "3b_o_m2048": (2048, 3072, 3072, "res"),
          "3b_gateup_m2048": (2048, 16384, 3072, "silu"), "3b_down_m2048": (2048, 3072, 8192, "res"),
          "7b_qkv_m128": (128, 12288, 4096, "bf16"), "7b_o_m128": (128, 4096, 4096, "res"),
          "7b_gateup_m128": (128, 22016, 4096, "silu"), "7b_down_m128": (128, 4096, 11008, "res"),
          "7b_qkv_m300": (300, 12288, 4096, "bf16"), "7b_o_m300": (300, 4096, 4096, "res"),
          "7b_down_m300": (300, 4096, 11008, "res"), "7b_o_m1024": (1024, 4096, 4096, "res"),
          "7b_down_m1024": (1024, 4096, 11008, "res"), "3b_o_m512": (512, 3072, 3072, "res")}
names = sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1] else list(SHAPES)
dev = torch.device("cuda:0")
flush = torch.empty(128 << 20, device=dev)
ext = ops.ext()


def timed(fn, cold):
    if cold:
        flush.fill_(1.0)
    else:
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000


for name in names:
    M, N, K, epi = SHAPES[name]
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16).to(dev)
    pw = ops.PackedWeight.from_dense(w)
    out = torch.zeros(M, N // 2 if epi == "silu" else N, device=dev,
                      dtype=torch.float32 if epi in ("f32", "res") else torch.bfloat16)
    table = ops.sk_config(M, N, K, epi)
    res = {}
    for cfg in sorted({table, 4, 5, 12, 13}):
        for mode in ("warm", "cold"):
            t = {0: [], 1: []}
            for _ in range(7):
                for one in (0, 1):
                    ext.gemm_sk_one_phase(one)
                    t[one].append(timed(lambda: ops.gemm_sk(x, pw.data, N, out, epi, cfg=cfg), mode == "cold"))
            ext.gemm_sk_one_phase(1)  # the default
            res[f"cfg{cfg}_{mode}"] = {"four_phase": round(st.median(t[0]), 1), "one_phase": round(st.median(t[1]), 1)}
    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "epi": epi, "table_cfg": table, **res}), flush=True)

"""The prefill qkv projection with the RoPE + paged-KV append epilogue (ops.linear_rope) under forced stream-K tile
configurations, next to the unfused route (bf16 GEMM with the table's configuration, then rope_append), on the 3B /
7B qkv shapes below ops.ROPE_FUSED_MIN_M.  us per call, interleaved rounds, hot weights.
    python scripts/rope_cfg_sweep.py [3b_2k,7b_4k,...] > gpurun_out/rope_cfg_sweep.jsonl
"""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.ops import reference as ref  # noqa: E402
from attn_scaling import timeit  # noqa: E402

dev = "cuda:0"
cos, sin = (t.to(dev) for t in ref.rope_tables(128, 8192, 500000.0, None))


def case(name, T, d, H, Hkv):
    N = (H + 2 * Hkv) * 128
    x = (torch.rand(T, d, device=dev) * 2 - 1).to(torch.bfloat16)
    pw = ops.PackedWeight.from_dense(((torch.rand(N, d, device=dev) * 2 - 1) / math.sqrt(d)).to(torch.bfloat16))
    nblk = (T + 63) // 64 + 1
    kc = torch.zeros(nblk + 1, Hkv, 64, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    bt = (torch.arange(nblk, device=dev, dtype=torch.int32) + 1).view(1, nblk)
    pos = torch.arange(T, device=dev, dtype=torch.int32)
    tsq = torch.zeros(T, device=dev, dtype=torch.int32)
    q = torch.empty(T, H, 128, device=dev, dtype=torch.bfloat16)
    qkv = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    ws, tk, ncu = ops._sk_workspace(dev)
    res = {"case": name, "T": T, "N": N, "K": d, "table_bf16_cfg": ops.sk_config(T, N, d, "bf16")}

    def unfused():
        ops.linear(x, pw, "bf16", out=qkv)
        ops.rope_append(qkv, pos, tsq, bt, cos, sin, q, kc, vc, H, Hkv)

    arms = {"unfused": unfused}
    for cfg in (-1, 0, 3, 8, 11, 16 + 0, 16 + 3, 16 + 8, 16 + 11):  # + 16: direct epilogue instead of the LDS image
        arms[f"rope_cfg{cfg}"] = (lambda c: lambda: ops.ext().gemm_sk_rope(
            x, pw.data, ws, tk, ncu, ops.SK_MIN_SHARE, c, pos, tsq, bt, cos, sin, q, kc, vc, H, Hkv))(cfg)
    for _ in range(2):
        for a, fn in arms.items():
            try:
                res.setdefault(a, []).append(round(timeit(fn), 2))
            except RuntimeError as e:  # a configuration the epilogue refuses
                res[a] = str(e)[:80]
    print(json.dumps(res), flush=True)


shapes = {"3b_2k": (2048, 3072, 24, 8), "3b_1k": (1024, 3072, 24, 8), "7b_2k": (2048, 4096, 32, 32),
          "7b_300": (300, 4096, 32, 32), "7b_4k": (4096, 4096, 32, 32), "3b_4k": (4096, 3072, 24, 8),
          "7b_8k": (8192, 4096, 32, 32)}
for nm in (sys.argv[1].split(",") if len(sys.argv) > 1 else list(shapes)[:4]):
    case(nm, *shapes[nm])

"""Which data k-positions each lane's E8M0 scale byte governs in v_mfma_scale_f32_16x16x128_f8f6f4, as driven by
ops.linear_a8 (csrc/kernels/gemm_fp8a.hip): one-hot weights W[n][k] = [k == n] (N = K = 128), activations all 1.0,
and one lane group's scale raised by one binade -- y[n] = 2 exactly where the raised scale covers data k = n.

  B side (activation scales, s8): fp8 and MXFP4 weights.   A side (MXFP4 weight scales): raised per lane group.
Prints one JSON line per probe: {"side", "wkind", "lane_group", "k_doubled": [...]}.
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
N = K = 128
w = torch.eye(N, K, device=dev).to(torch.bfloat16)
x = torch.ones(1, K, device=dev).to(torch.bfloat16)
x8, sx = ops.quantize_xf8(x)  # 1.0 = 448 * (1 / 448): every byte the same e4m3 code
for wkind in ("fp8", "mxfp4"):
    pw = ops.PackedWeight.from_dense(w, wkind)
    for gs in range(4):
        s8 = torch.full((64,), 127, dtype=torch.uint8, device=dev)
        s8[16 * gs: 16 * gs + 16] = 128
        y = ops.linear_a8(x8, sx, 1, pw, "f32", s8=s8)[0, 0]
        ratio = (y / y.max().clamp(min=1e-30)).cpu()
        print(json.dumps({"side": "B", "wkind": wkind, "lane_group": gs,
                          "k_doubled": [int(k) for k in torch.nonzero(ratio > 0.75).flatten()],
                          "y_unique": sorted(set(round(float(v), 4) for v in y.cpu()))}), flush=True)
pw = ops.PackedWeight.from_dense(w, "mxfp4")
base = pw.scale.clone()
for gs in range(4):
    sc = base.clone()
    v = sc.view(N // 16, -1, 64, 4)  # [nb][kb4][lane][4 kb]
    v[:, :, 16 * gs: 16 * gs + 16, 0] += 1
    pw.scale = sc
    s8 = torch.full((64,), 127, dtype=torch.uint8, device=dev)
    y = ops.linear_a8(x8, sx, 1, pw, "f32", s8=s8)[0, 0]
    ratio = (y / y.max().clamp(min=1e-30)).cpu()
    print(json.dumps({"side": "A", "wkind": "mxfp4", "lane_group": gs,
                      "k_doubled": [int(k) for k in torch.nonzero(ratio > 0.75).flatten()],
                      "y_unique": sorted(set(round(float(v), 4) for v in y.cpu()))}), flush=True)

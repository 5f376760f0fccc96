"""MXFP4 weight quantisation (ops.quantize_mxfp4 / pack_mxfp4 / dequantize_mxfp4), CPU: the OCP MX rules the GPU
kernels (csrc/kernels/gemm_fp4.hip) rely on -- e2m1 grid values, power-of-two block scales, the nibble / lane /
scale-word layout -- and the CPU engine path of an mxfp4 model (its weights are the dequantised values)."""
import torch

from llm_based_apache_spark_optimization_amd import ops
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import init_random


def test_quantize_values_on_the_e2m1_grid_with_power_of_two_scales():
    torch.manual_seed(0)
    w = torch.randn(32, 256) * torch.logspace(-3, 1, 32)[:, None]
    codes, sb = ops.quantize_mxfp4(w)
    assert codes.dtype == torch.uint8 and int(codes.max()) <= 15
    d = ops.dequantize_mxfp4(*ops.pack_mxfp4(codes, sb), 32, 256)
    scale = torch.exp2(sb.float() - 127).repeat_interleave(32, 1)
    grid = torch.tensor(ops.FP4_VALUES)
    q = (d / scale).abs()
    assert torch.isin(q, grid).all()  # every element is an e2m1 value times its block's 2^e
    # OCP MX: the block's largest magnitude lands in [4, 6] after scaling (floor(log2 amax) - 2, saturated at 6)
    amax = w.abs().view(32, 8, 32).amax(-1)
    top = (amax / torch.exp2(sb.float() - 127))
    assert ((top >= 4) & (top < 8)).all()
    assert float((d - w).norm() / w.norm()) < 0.15


def test_pack_layout_matches_the_kernel_contract():
    N, K = 32, 640  # K / 128 = 5: the scale words are padded to 8 steps
    codes = torch.randint(0, 16, (N, K), dtype=torch.uint8)
    sb = torch.randint(100, 140, (N, K // 32), dtype=torch.uint8)
    wq, sw = ops.pack_mxfp4(codes, sb)
    assert wq.shape == (N // 16, K // 128, 64, 16) and sw.shape == (N // 16, 2, 64, 4)
    # lane 16 g + r of (nb, kb) holds row 16 nb + r, k = 128 kb + 32 g + 2 i (low nibble) / 2 i + 1 (high nibble)
    nb, kb, g, r, i = 1, 3, 2, 5, 7
    byte = int(wq[nb, kb, 16 * g + r, i])
    row, k = 16 * nb + r, 128 * kb + 32 * g + 2 * i
    assert byte & 15 == int(codes[row, k]) and byte >> 4 == int(codes[row, k + 1])
    # the lane's scale word: byte kb % 4 of word kb // 4 is the block (row, 4 kb + g)
    assert int(sw[nb, kb // 4, 16 * g + r, kb % 4]) == int(sb[row, 4 * kb + g])
    vals = torch.tensor(ops.FP4_VALUES)[codes.long() & 7] * (1 - 2 * (codes.long() >> 3).float())
    exp = (vals.view(N, K // 32, 32) * torch.exp2(sb.float() - 127)[..., None]).view(N, K)
    assert torch.equal(ops.dequantize_mxfp4(wq, sw, N, K), exp)


def test_zero_block_and_cpu_model():
    codes, sb = ops.quantize_mxfp4(torch.zeros(16, 128))
    assert int(sb.max()) == 0 and torch.equal(ops.dequantize_mxfp4(*ops.pack_mxfp4(codes, sb), 16, 128),
                                             torch.zeros(16, 128))
    # on the CPU the model keeps dense weights (the reference path); kind="mxfp4" is a GPU weight format
    w = init_random(get_spec("tiny-nsql"), "cpu", seed=0, kind="mxfp4")
    assert w.layers[0].wqkv.kind == "dense"

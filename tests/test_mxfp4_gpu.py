"""MXFP4 W4A16 GEMMs (csrc/kernels/gemm_fp4.hip) against a plain fp32 PyTorch product over the dequantised
weights, the prefill dequantisation kernel bit for bit, and an mxfp4 engine against its fp32 oracle."""
import math

import pytest
import torch

from llm_based_apache_spark_optimization_amd import ops
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine
from llm_based_apache_spark_optimization_amd.eval import numerics as nm
from llm_based_apache_spark_optimization_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp(min=1e-12))


def test_fp4_dequant_kernel_exact(gpu):
    torch.manual_seed(0)
    N, K = 96, 1408  # K / 128 = 11: padded scale words
    w = torch.randn(N, K, device=gpu) * 0.05
    pw = ops.PackedWeight.from_dense(w, "mxfp4")
    buf = torch.empty(N * K, device=gpu, dtype=torch.bfloat16)
    ops.ext().fp4_dequant(pw.data, pw.scale, N, K, buf)
    got = ops.unshuffle_weight(buf, N, K).float()
    assert torch.equal(got, ops.dequantize_mxfp4(pw.data, pw.scale, N, K))


@pytest.mark.parametrize("M", [1, 5, 16, 20, 32, 40, 64, 130])
@pytest.mark.parametrize("epi", ["bf16", "f32", "silu"])
def test_fp4_gemm(gpu, M, epi):
    N, K = 1024, 4096
    torch.manual_seed(M)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(torch.bfloat16)
    pw = ops.PackedWeight.from_dense(w, "mxfp4")
    wd = ops.dequantize_mxfp4(pw.data, pw.scale, N, K)
    yr = ref.linear(x, wd, epi)
    for nb, sk, waves in ((1, 1, 4), (2, 2, 8), (4, 4, 4)):
        if epi != "f32" and sk > 1:
            sk = 1
        if epi == "silu" and nb < 2:
            nb = 2
        y = ops.linear(x, pw, epi, splitk=sk, nb=nb, waves=waves)
        if epi == "f32":
            y = y.sum(0)
        assert _rel(y, yr) < 1e-2, (M, epi, nb, sk, waves)
        if M <= 64:  # fragment-major activations (the decode path at B > 16)
            yx = ops.linear_xf(ops.to_xfrag(x), M, pw, epi, splitk=sk, nb=nb, waves=waves)
            if epi == "f32":
                yx = yx.sum(0)
            elif epi == "silu":
                yx = ops.from_xfrag(yx, M, N // 2)
            assert _rel(yx, yr) < 1e-2, (M, epi, nb, sk, waves, "xf")


@pytest.mark.parametrize("M", [1, 16, 32])
def test_fp4_gemm_norm_free_epilogues(gpu, M):
    """rownorm (row scale rsqrt(ss / K + eps)) and the residual epilogue (h += y, bf16 x, row sums of squares)."""
    N, K = 512, 2048
    torch.manual_seed(7)
    x = (torch.randn(M, K, device=gpu) * 3).to(torch.bfloat16)
    pw = ops.PackedWeight.from_dense(torch.randn(N, K, device=gpu) / math.sqrt(K), "mxfp4")
    wd = ops.dequantize_mxfp4(pw.data, pw.scale, N, K)
    ss = ops.ss_q24(x.float().pow(2).sum(1))
    y = ops.linear(x, pw, "f32", splitk=1, rownorm=(ss, 1e-5))[0]
    xs = x.float() * torch.rsqrt(x.float().pow(2).sum(1, keepdim=True) / K + 1e-5)
    assert _rel(y, xs @ wd.t()) < 1e-2
    h0 = torch.randn(M, N, device=gpu)
    for sk in (1, 2):
        h, xo = h0.clone(), torch.zeros(M, N, device=gpu, dtype=torch.bfloat16)
        so = torch.zeros(M, device=gpu, dtype=torch.int64)
        tk = torch.zeros(N // 16, device=gpu, dtype=torch.int32)
        ops.linear(x, pw, "res", splitk=sk, res=(h, xo, so, tk))
        hr = h0 + x.float() @ wd.t()
        assert _rel(h, hr) < 1e-3, sk
        assert torch.allclose(ops.ss_float(so), hr.pow(2).sum(1), rtol=1e-3), sk


@pytest.mark.parametrize("batch", [2, 20])
def test_mxfp4_engine_numerics(gpu, batch):
    """An mxfp4 engine (prefill on dequantised bf16 weights, W4A16 decode) against the fp32 oracle over the same
    dequantised weights: teacher-forced KL / top-1 / top-5 over 32 decode steps."""
    eng = build_engine("tiny-nsql", device=str(gpu), dtype="mxfp4", max_slots=32, max_model_len=512, seed=1)
    assert eng.runner.w.layers[0].wqkv.kind == "mxfp4"
    g = torch.Generator().manual_seed(batch)
    prompts = [[1] + torch.randint(3, eng.spec.vocab_size, (30 + 3 * i,), generator=g).tolist() for i in range(batch)]
    res = nm.teacher_forced_check(eng, prompts, 32, check_rows=(0, batch - 1))
    assert res["ok"], res
    out = eng.generate(prompts[:2], SamplingParams(max_tokens=8, ignore_eos=True))
    assert all(r.eval_count == 8 for r in out)


def test_fp4_prefill_two_streams_match_serial(gpu):
    """Co-served MXFP4 engines prefill on their own streams (client.py): each stream has its own dequant scratch,
    so interleaved prefill GEMMs of two different models give the same results as serial runs."""
    torch.manual_seed(3)
    M, K = 256, 2048
    wa = ops.PackedWeight.from_dense(torch.randn(2048, K, device=gpu) / math.sqrt(K), "mxfp4")
    wb = ops.PackedWeight.from_dense(torch.randn(4096, K, device=gpu) / math.sqrt(K), "mxfp4")  # regrows the scratch
    xa = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    xb = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    ya0, yb0 = ops.linear(xa, wa, "bf16"), ops.linear(xb, wb, "bf16")
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(8):
        with torch.cuda.stream(sa):
            ya = ops.linear(xa, wa, "bf16")
        with torch.cuda.stream(sb):
            yb = ops.linear(xb, wb, "bf16")
        outs.append((ya, yb))
    torch.cuda.synchronize()
    for ya, yb in outs:
        assert torch.equal(ya, ya0) and torch.equal(yb, yb0)

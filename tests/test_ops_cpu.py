"""CPU checks of the op-level layout helpers and the fragment-major (xf) paths of the fp32 oracle."""
import math

import torch

from llm_based_apache_spark_optimization_amd import ops
from llm_based_apache_spark_optimization_amd.ops import reference as ref


def test_xfrag_roundtrip_and_index():
    for M in (1, 16, 17, 32, 48, 64):
        x = torch.randn(M, 128).to(torch.bfloat16)
        xf = ops.to_xfrag(x)
        mt = ops.xfrag_tiles(M)
        assert xf.numel() == mt * 16 * 128
        assert torch.equal(ops.from_xfrag(xf, M, 128), x)
        # the element-offset formula the HIP kernels use (common.h xf_off)
        for m, k in ((0, 0), (M - 1, 127), (M // 2, 37)):
            off = (((k // 32) * mt + m // 16) * 64 + 16 * ((k % 32) // 8) + m % 16) * 8 + k % 8
            assert xf[off] == x[m, k]
        # padding rows are zero
        full = xf.view(128 // 32, mt, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(mt * 16, 128)
        assert not full[M:].any()


def test_linear_xf_cpu_matches_linear():
    torch.manual_seed(0)
    M, K, N = 20, 256, 64
    x = torch.randn(M, K).to(torch.bfloat16)
    w = (torch.randn(N, K) / math.sqrt(K)).to(torch.bfloat16)
    pw = ops.PackedWeight.from_dense(w)
    y = ops.linear_xf(ops.to_xfrag(x), M, pw, "f32")
    assert torch.allclose(y.sum(0), ops.linear(x, pw, "f32").sum(0))
    gu = ops.PackedWeight.from_dense(ops.interleave_gate_up(w[:32], w[32:]))
    ys = ops.linear_xf(ops.to_xfrag(x), M, gu, "silu")
    assert torch.equal(ops.from_xfrag(ys, M, 32), ops.linear(x, gu, "silu"))


def test_norm_and_attention_xf_cpu():
    torch.manual_seed(1)
    rows, D = 18, 64
    h = torch.randn(rows, D)
    w = torch.randn(D).to(torch.bfloat16)
    xr = torch.empty(rows, D, dtype=torch.bfloat16)
    ops.add_rmsnorm(h.clone(), w, 1e-5, xr)
    xf = torch.zeros(ops.xfrag_tiles(rows) * 16 * D, dtype=torch.bfloat16)
    ops.add_rmsnorm(h.clone(), w, 1e-5, xf, rows=rows, xf=True)
    assert torch.equal(ops.from_xfrag(xf, rows, D), xr)
    # attention: 2 sequences, 1 kv head, 1 block each
    H, Hkv, Dh = 2, 1, 128
    kc = torch.randn(3, Hkv, 64, Dh).to(torch.bfloat16)
    vc = torch.randn(3, Hkv, 64, Dh).to(torch.bfloat16)
    bt = torch.tensor([[1], [2]], dtype=torch.int32)
    pos = torch.tensor([5, 63], dtype=torch.int32)
    q = torch.randn(2, H, Dh).to(torch.bfloat16)
    o = torch.empty(2, H, Dh, dtype=torch.bfloat16)
    ref.attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.1, o)
    of = torch.zeros(16 * H * Dh, dtype=torch.bfloat16)
    ops.attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.1, of, xf=True)
    assert torch.equal(ops.from_xfrag(of, 2, H * Dh), o.view(2, -1))


def _check_plan(cu, ctx, heads, monkeypatch, split):
    monkeypatch.setattr(ops, "PREFILL_SPLIT", split)
    work, combine, npl = ops.prefill_plan_items(cu, ctx=ctx, kernel="32", heads=heads)
    units = [tuple(w[i:i + 5]) for w in work for i in range(0, len(w), 5) if w[i] >= 0]
    cover = {}
    for s, qs, t0, t1, ps in units:
        assert 0 <= t0 < t1
        cover.setdefault((s, qs), []).append((t0, t1, ps))
    merges = {(s, qs): (p0, k) for s, qs, p0, k in combine}
    for w in work:  # in-workgroup halves: both groups of the row on one block, nowhere else
        if len(w) == 10 and w[4] == -2:
            assert w[9] == -2 and (w[0], w[1]) == (w[5], w[6]) and w[3] == w[7]
    slots = []
    for s in range(len(cu) - 1):
        ql, pos0 = cu[s + 1] - cu[s], ctx[s] - (cu[s + 1] - cu[s])
        for qs in range(0, ql, 128):
            nt = (pos0 + min(qs + 128, ql) + 63) // 64
            pieces = sorted(cover.pop((s, qs)))
            assert pieces[0][0] == 0 and pieces[-1][1] == nt  # every causal key tile exactly once
            assert all(a[1] == b[0] for a, b in zip(pieces, pieces[1:]))
            if len(pieces) == 1:
                assert pieces[0][2] == -1 and (s, qs) not in merges
            elif pieces[0][2] == -2:
                assert len(pieces) == 2 and pieces[1][2] == -2 and (s, qs) not in merges
            else:
                p0, k = merges.pop((s, qs))
                assert k == len(pieces) and sorted(p[2] for p in pieces) == list(range(p0, p0 + k))
                slots += [p[2] for p in pieces]
    assert not cover and not merges and sorted(slots) == list(range(npl))
    return units, npl


def test_prefill_plan_kv_splits_cover_causal_ranges(monkeypatch):
    """ops.prefill_plan for the 32-row kernel: each query block's causal key tiles are covered exactly once by
    its pieces, split blocks get consecutive partial slots and one merge row, unsplit blocks write directly."""
    monkeypatch.setattr(ops, "PREFILL_PAIR", "auto")
    # 2k prompt (3B heads): the auto budget splits the heavy half of the blocks
    units, npl = _check_plan([0, 2048], [2048], 24, monkeypatch, "auto")
    assert npl > 0 and max(t1 - t0 for _, _, t0, t1, _ in units) <= ops._split_tiles(272 * 24)
    # chunked continuation and several sequences, forced small budget; and splitting off
    _check_plan([0, 10, 210, 310], [700, 264, 400], 32, monkeypatch, "3")
    monkeypatch.setattr(ops, "PREFILL_HALVES", "0")
    _, npl = _check_plan([0, 2048], [2048], 24, monkeypatch, "0")
    assert npl == 0
    # in-workgroup halves (no splits): every block of >= 2 tiles is one workgroup row of two halves
    monkeypatch.setattr(ops, "PREFILL_HALVES", "auto")  # (opt-in: the default is "0")
    units, npl = _check_plan([0, 2048], [2048], 24, monkeypatch, "0")
    assert npl == 0 and len(units) == 32 and all(ps == -2 for *_, ps in units)
    _check_plan([0, 10, 210, 310], [700, 264, 400], 32, monkeypatch, "0")
    # an 8k prompt already has more blocks than slots: no splits under auto
    _, npl = _check_plan([0, 8192], [8192], 24, monkeypatch, "auto")
    assert npl == 0

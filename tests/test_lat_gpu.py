"""Latency-path kernels (csrc/kernels/decode_lat.hip) against plain fp32 PyTorch, and the batch-<=4 engine path
against the fp32 oracle at production shapes."""
import dataclasses
import math

import pytest
import torch

from llm_based_apache_spark_optimization_amd import ops
from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner, SamplingParams
from llm_based_apache_spark_optimization_amd.eval import numerics as nm
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import init_random

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp(min=1e-12))


def _w(N, K, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    w = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(torch.bfloat16)
    return w, ops.PackedWeight.from_dense(w)


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("N,K,nb,sk", [(5120, 3072, 1, 2), (12288, 4096, 2, 2), (1024, 4096, 4, 8), (512, 2048, 8, 1)])
def test_lat_hq_f32(gpu, M, N, K, nb, sk):
    """src hq (Q32 stream, row sums published in-kernel) -> f32 split-K slabs, rows RMS-scaled."""
    torch.manual_seed(M + N)
    h = torch.randn(M, K, device=gpu) * 3
    hq = ops.to_q32(h)
    w, pw = _w(N, K, gpu, N + K)
    ss = torch.zeros(8, dtype=torch.int64, device=gpu)
    out = torch.empty(sk, M, N, device=gpu)
    st = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.lat_linear(pw, M, "hq", "f32", sk, nb, 4, hq=hq, ss=ss, eps=1e-5, out=out, stats=st)
    hf = ops.from_q32(hq)
    want = (hf.to(torch.bfloat16).float() @ w.float().t()) * torch.rsqrt(hf.pow(2).mean(1, keepdim=True) + 1e-5)
    assert _rel(out.sum(0), want) < 2e-3
    assert int(st) == 0  # every row-sum poll found all publishers
    assert [int(v) & 255 for v in ss[:M].tolist()] == [sk] * M


@pytest.mark.parametrize("M", [1, 4])
@pytest.mark.parametrize("waves", [4, 8])
def test_lat_hq_silu(gpu, M, waves):
    torch.manual_seed(M)
    N, K = 2 * 8192, 3072
    h = torch.randn(M, K, device=gpu)
    hq = ops.to_q32(h)
    wg, _ = _w(N // 2, K, gpu, 1)
    wu, _ = _w(N // 2, K, gpu, 2)
    pw = ops.PackedWeight.from_dense(ops.interleave_gate_up(wg, wu))
    ss = torch.zeros(4, dtype=torch.int64, device=gpu)
    act = torch.empty(M, N // 2, device=gpu, dtype=torch.bfloat16)
    ops.lat_linear(pw, M, "hq", "silu", 1, 2, waves, hq=hq, ss=ss, eps=1e-5, act=act)
    x = ops.from_q32(hq)
    rs = torch.rsqrt(x.pow(2).mean(1, keepdim=True) + 1e-5)
    xb = x.to(torch.bfloat16).float()
    want = torch.nn.functional.silu((xb @ wg.float().t()) * rs) * ((xb @ wu.float().t()) * rs)
    assert _rel(act, want) < 5e-3


@pytest.mark.parametrize("M", [1, 3])
@pytest.mark.parametrize("N,K,nb,sk", [(3072, 8192, 2, 4), (4096, 11008, 2, 4), (4096, 4096, 8, 1)])
def test_lat_act_atom(gpu, M, N, K, nb, sk):
    """src act (bf16 rows) -> Q32 integer atomics into the residual stream."""
    torch.manual_seed(K + M)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    w, pw = _w(N, K, gpu, 7)
    h0 = torch.randn(M, N, device=gpu)
    hq = ops.to_q32(h0)
    ops.lat_linear(pw, M, "act", "atom", sk, nb, 4, x=x, hq_out=hq)
    want = h0 + x.float() @ w.float().t()
    assert _rel(ops.from_q32(hq) - h0, want - h0) < 1e-4
    # integer adds: the same call again lands on exactly the same bits regardless of arrival order
    hq2 = ops.to_q32(h0)
    ops.lat_linear(pw, M, "act", "atom", sk, nb, 4, x=x, hq_out=hq2)
    assert torch.equal(hq, hq2)


@pytest.mark.parametrize("M,H,ctx", [(1, 24, 2100), (1, 32, 200), (4, 32, 130), (2, 24, 64)])
def test_lat_part_atom(gpu, M, H, ctx):
    """src part: the o projection merges split-KV partials (o unnormalised, (m, l) in the log2 domain) of its heads."""
    torch.manual_seed(H + ctx)
    nsplit = (ctx + 63) // 64 + 2  # a plan wider than the context: splits past nse are never read
    plan = (1, nsplit, 0)
    pos = torch.tensor([ctx - 1 - 3 * i for i in range(M)], dtype=torch.int32, device=gpu)
    opart = torch.randn(M, H, nsplit, 128, device=gpu)
    mvals = torch.randn(M, H, nsplit, device=gpu) * 2
    lvals = torch.rand(M, H, nsplit, device=gpu) * 5 + 0.5
    ml = torch.stack([mvals, lvals], -1).contiguous()  # float pairs (m, l) = u64 (l << 32 | m)
    N, K = 1024, H * 128
    w, pw = _w(N, K, gpu, 3)
    h0 = torch.randn(M, N, device=gpu)
    hq = ops.to_q32(h0)
    ops.lat_linear(pw, M, "part", "atom", H, 8, 4, part=(opart, ml, pos, plan, H), hq_out=hq)
    x = torch.empty(M, H, 128, device=gpu)
    for m in range(M):
        nse = (int(pos[m]) + 1 + 63) // 64
        mm, ll, oo = mvals[m, :, :nse], lvals[m, :, :nse], opart[m, :, :nse]
        wt = torch.exp2(mm - mm.max(1, keepdim=True).values)
        x[m] = (oo * wt[..., None]).sum(1) / (ll * wt).sum(1, keepdim=True)
    want = x.reshape(M, K).to(torch.bfloat16).float() @ w.float().t()
    assert _rel(ops.from_q32(hq) - h0, want) < 2e-3


def _lat_engine(gpu, model, layers, lat=True, kv="bf16"):
    spec = dataclasses.replace(get_spec(model), n_layers=layers, name=f"{model}-{layers}l")
    w = init_random(spec, gpu, seed=5, kind="bf16")
    r = ModelRunner(w, max_slots=8, max_model_len=2560, use_graphs=True, num_kv_blocks=8 * 40 + 1, lat=lat,
                    kv_dtype=kv)
    return LLMEngine(r, name=spec.name)


@pytest.mark.parametrize("model", ["duckdb-nsql", "llama3.2"])
@pytest.mark.parametrize("B", [1, 4])
def test_lat_engine_numerics(gpu, model, B):
    """The latency path at production shapes (4 layers) against the fp32 oracle, teacher-forced over 64 steps, with
    a context long enough for many attention splits per head, and no row-sum poll fallbacks."""
    eng = _lat_engine(gpu, model, 4)
    assert eng.runner.lat
    g = torch.Generator().manual_seed(11)
    prompts = [[1] + torch.randint(3, 30000, (700 + 300 * i,), generator=g).tolist() for i in range(B)]
    res = nm.teacher_forced_check(eng, prompts, 64, check_rows=(0, B - 1) if B > 1 else (0,))
    assert res["ok"], res
    assert int(eng.runner.lat_stats) == 0


def test_lat_engine_matches_general_path(gpu):
    """Greedy tokens of the latency path == the general decode step's (same weights, batch 1 and 3)."""
    a = _lat_engine(gpu, "llama3.2", 2, lat=True)
    b = _lat_engine(gpu, "llama3.2", 2, lat=False)
    g = torch.Generator().manual_seed(5)
    prompts = [[1] + torch.randint(3, 30000, (60 + 500 * i,), generator=g).tolist() for i in range(3)]
    sp = SamplingParams(max_tokens=24, ignore_eos=True)
    for B in (1, 3):
        ta = [r.token_ids for r in a.generate(prompts[:B], sp)]
        tb = [r.token_ids for r in b.generate(prompts[:B], sp)]
        agree = sum(x == y for p, q in zip(ta, tb) for x, y in zip(p, q)) / sum(len(p) for p in ta)
        assert agree > 0.9, (B, ta, tb)

"""Engine numerics at PRODUCTION shapes ("what's weak" 6): duckdb-nsql-7B and
Llama-3.2-3B at their real hidden/head/ffn/vocab dims (2 layers, random init), bf16 and fp8 weights,
decode batches 1 / 20 / 32 so the skinny GEMM, the fragment-major (xf) path and the tuned table entries
that ``bench.py`` times are the ones checked, with captured hipGraphs, against the plain fp32 PyTorch
forward over the same packed weights (``models.llama.reference_forward``; fp8 models are compared with
their own dequantised weights, so the tolerance measures the kernels, not the quantiser).

Checks: (1) prefill last-position logits of a packed multi-sequence prefill (the 256² tile GEMM and
the prefill attention) against the oracle; (2) every greedily decoded token, teacher-forced through the
oracle, is within a bf16-noise margin of the oracle's argmax.
"""
import dataclasses

import pytest
import torch

from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner, SamplingParams
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import init_random, reference_forward

pytestmark = pytest.mark.gpu

_CACHE = {}


def _engine(gpu, model, dtype):
    key = (model, dtype)
    if key not in _CACHE:
        _CACHE.clear()
        torch.cuda.empty_cache()
        spec = dataclasses.replace(get_spec(model), n_layers=2, name=f"{model}-2l")
        w = init_random(spec, gpu, seed=11, kind=dtype)
        runner = ModelRunner(w, max_slots=64, max_model_len=512, use_graphs=True)
        _CACHE[key] = LLMEngine(runner, name=spec.name)
    return _CACHE[key]


def _prompts(V, n, seed):
    g = torch.Generator().manual_seed(seed)
    return [[1] + torch.randint(3, min(V, 30000), (int(40 + 13 * i % 170),), generator=g).tolist() for i in range(n)]


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("model", ["duckdb-nsql", "llama3.2"])
def test_prefill_logits_prod_shapes(gpu, model, dtype):
    eng = _engine(gpu, model, dtype)
    r = eng.runner
    prompts = _prompts(r.V, 6, 1)
    for i in range(len(prompts)):
        r.set_slot(i, list(range(1 + 8 * i, 9 + 8 * i)), 4)
    r.prefill([(i, p, 0) for i, p in enumerate(prompts)])
    ours = r.logits_l[: len(prompts)].float()
    for i, p in enumerate(prompts):
        ref = reference_forward(r.w, p, act_quant_rows=len(p))[-1]  # packed prefill > 64 rows: W8A8 if fp8
        rel = ((ours[i] - ref).norm() / ref.norm()).item()
        # fp8: the prefill runs W8A8 (per-token e4m3 activations).  The oracle applies the same rounding, but
        # activations that sit near an e4m3 rounding boundary round differently from the oracle's (bf16-level
        # differences vs a 6-12 % ulp), so ~5-7 % logit error remains at 2 layers (bf16: < 1 %)
        assert rel < (1e-1 if dtype == "fp8" else 2e-2), (model, dtype, i, rel)
    for i in range(len(prompts)):
        r.release_slot(i)


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("model", ["duckdb-nsql", "llama3.2"])
@pytest.mark.parametrize("B", [1, 20, 32, 48])
def test_decode_tokens_prod_shapes(gpu, model, dtype, B):
    eng = _engine(gpu, model, dtype)
    prompts = _prompts(eng.runner.V, B, 100 + B)
    assert eng.runner.use_xfrag(eng.runner.bucket(B)) == (B > 16)
    res = eng.generate(prompts, SamplingParams(max_tokens=12, ignore_eos=True))
    worst = 0.0
    for p, out in zip(prompts, res[: min(B, 6)] if B > 1 else res):
        rows = sum(len(q) for q in prompts)  # one packed prefill: W8A8 for fp8 weights when > 64 rows
        # decode buckets of an fp8 model run some projections W8A8 (ops.linear_a8, ModelRunner.a8_plan)
        r, bk = eng.runner, eng.runner.bucket(B)
        lg = reference_forward(r.w, p + out.token_ids[:-1], act_quant_rows=len(p) if rows > 64 else 0,
                               decode_a8=r.oracle_plan(bk))[len(p) - 1:]
        chosen = lg.gather(1, torch.tensor(out.token_ids, device=lg.device).view(-1, 1)).squeeze(1)
        top = lg.max(1).values
        spread = lg.std(1)
        gap = ((top - chosen) / spread).max().item()  # in units of the logit spread
        worst = max(worst, gap)
    assert worst < 0.15, (model, dtype, B, worst)

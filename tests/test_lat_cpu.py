"""Batch-<=4 latency decode path (csrc/kernels/decode_lat.hip, engine/runner.py _decode_step_lat) on the CPU: the
ops' reference semantics (Q32 residual stream, folded norms with row sums, partial-merging o projection) decode the
same greedy tokens as the general decode step, and the fp32 oracle agrees."""
import torch

from llm_based_apache_spark_optimization_amd import ops
from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner, SamplingParams
from llm_based_apache_spark_optimization_amd.eval import numerics as nm
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import init_random


def _eng(model, lat):
    w = init_random(get_spec(model), "cpu", seed=2)
    return LLMEngine(ModelRunner(w, max_slots=8, max_model_len=512, lat=lat), name=model)


def test_lat_path_matches_general_step():
    for model in ("tiny-nsql", "tiny-llama3"):
        a, b = _eng(model, True), _eng(model, False)
        assert a.runner.lat and not b.runner.lat
        prompts = [[1] + list(range(5, 5 + n)) for n in (9, 70, 33)]
        sp = SamplingParams(max_tokens=12, ignore_eos=True)
        for B in (1, 3):
            ta = [r.token_ids for r in a.generate(prompts[:B], sp)]
            tb = [r.token_ids for r in b.generate(prompts[:B], sp)]
            assert ta == tb, (model, B)


def test_lat_path_numerics_vs_oracle():
    eng = _eng("tiny-nsql", True)
    res = nm.teacher_forced_check(eng, [[1] + list(range(9, 60))], 16)
    assert res["ok"] and res["mean_kl"] < 1e-4, res


def test_q32_roundtrip():
    v = torch.tensor([1.5, -2.25, 1e-6, -3e4, 0.0])
    assert torch.allclose(ops.from_q32(ops.to_q32(v)), v, rtol=1e-6, atol=3e-10)

"""The bench's decode numerics check (eval/numerics.py) must be able to FAIL.

A 4-layer duckdb-nsql-7B-shaped engine (production hidden / head / ffn / vocab dims, random init) and a 4-layer
Llama-3.2-3B-shaped one (GQA 3:1, tied lm_head: checked through the final hidden state and a random probe head,
eval/numerics.py TIED_THRESHOLDS) decode a batch for 64 steps; the teacher-forced comparison against the fp32 oracle passes at HEAD and fails when a
fault is injected into the ENGINE only (the oracle keeps the true weights / cache semantics):

* one layer's down-projection weight scale x1.25 (fp8) / weights x1.25 (bf16) / every 8th E8M0 block scale one
  binade up (MXFP4, decoded W4A8: e2m1 weights + E8M0 scales straight into the block-scaled MFMA): a wrong
  dequantisation scale;
* a swapped token pair in the K cache layout (keys of positions 2k and 2k + 1 exchanged in the first block of
  every layer after prefill, values left in place): a KV layout bug.
"""
import dataclasses

import pytest
import torch

from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner
from llm_based_apache_spark_optimization_amd.eval import numerics as nm
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import init_random

pytestmark = pytest.mark.gpu

SPEC = dataclasses.replace(get_spec("duckdb-nsql"), n_layers=4, name="duckdb-nsql-4l")
# Llama-3.2-3B shape (GQA 3:1, TIED lm_head): the check runs on the final hidden state through a random probe head
SPEC3B = dataclasses.replace(get_spec("llama3.2"), n_layers=4, name="llama3.2-4l")


def _engine(gpu, dtype, kv, spec=SPEC):
    w = init_random(spec, gpu, seed=5, kind=dtype)
    r = ModelRunner(w, max_slots=32, max_model_len=512, use_graphs=True, num_kv_blocks=32 * 8 + 1, kv_dtype=kv)
    return LLMEngine(r, name=spec.name)


def _prompts(n, seed=3):
    g = torch.Generator().manual_seed(seed)
    return [[1] + torch.randint(3, 30000, (100 + 7 * i,), generator=g).tolist() for i in range(n)]


def _check(eng, B, weights=None):
    return nm.teacher_forced_check(eng, _prompts(B), 64, check_rows=(0, B - 1) if B > 1 else (0,), weights=weights)


@pytest.mark.parametrize("dtype,kv", [("bf16", "bf16"), ("fp8", "bf16"), ("fp8", "fp8"), ("mxfp4", "bf16")])
@pytest.mark.parametrize("model,B", [("7b", 4), ("7b", 32), ("3b", 1), ("3b", 4)])
def test_numerics_check_passes_and_catches_faults(gpu, dtype, kv, model, B):
    spec = SPEC if model == "7b" else SPEC3B
    eng = _engine(gpu, dtype, kv, spec)
    good = _check(eng, B)
    assert good["ok"] and good["tokens_checked"] >= 64, good
    if dtype == "mxfp4":  # qkv / gate_up run W4A8 at every bucket, o / down up to 16 rows (ModelRunner.a8_plan)
        assert eng.runner.a8_plan(B) == (True, True, B <= 16, B <= 16) and good["class"] == "w4a8", good
    if spec is SPEC3B:  # the tied head's own KL is degenerate (~0): the probe statistic must not be
        assert good["tied_head"] and good["probe_kl"] > 0, good

    # fault 1: a wrong weight scale in one layer of the engine (the oracle gets a fresh copy of the true weights)
    truth = init_random(spec, gpu, seed=5, kind=dtype)
    with nm.scale_fault(eng, 1, 1.25):
        bad_scale = _check(eng, B, weights=truth)
    assert not bad_scale["ok"], (good, bad_scale)

    # fault 2: keys of a token pair swapped in the cache layout (every layer, first block of every sequence)
    with nm.kv_swap_fault(eng):
        bad_kv = _check(eng, B, weights=truth)
    assert not bad_kv["ok"], (good, bad_kv)
    print({"good": good, "bad_scale": bad_scale, "bad_kv": bad_kv})

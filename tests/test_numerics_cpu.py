"""Tied-embedding numerics statistic on CPU (eval/numerics.py): with a random-init tied lm_head the head's own KL is
~0 whatever the layers compute, the probe-head statistic over the final hidden state is not, and an injected
weight-scale fault moves it past its bound."""
import torch

from llm_based_apache_spark_optimization_amd.engine import build_engine
from llm_based_apache_spark_optimization_amd.eval import numerics as nm
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import init_random


def test_tied_head_probe_statistic():
    eng = build_engine("tiny-llama3", device="cpu", max_slots=4, max_model_len=512)
    g = torch.Generator().manual_seed(3)
    ps = [[1] + torch.randint(3, 600, (40 + 7 * i,), generator=g).tolist() for i in range(2)]
    good = nm.teacher_forced_check(eng, ps, 32, check_rows=(0, 1))
    assert good["tied_head"] and good["ok"], good
    assert good["mean_kl"] < 1e-6 and good["probe_kl"] > 0  # the degenerate head vs the live statistic
    truth = init_random(get_spec("tiny-llama3"), "cpu", seed=0)
    with nm.scale_fault(eng, 1, 1.25):
        bad = nm.teacher_forced_check(eng, ps, 32, check_rows=(0, 1), weights=truth)
    assert not bad["ok"] and bad["probe_kl"] > 20 * good["probe_kl"], (good, bad)
    assert bad["mean_kl"] < 1e-6  # ... which the tied head's KL alone would have passed

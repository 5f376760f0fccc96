"""A served TP=2 replica behind the FastAPI app (BASELINE config 4's replica shape):
``LSA_TP=2`` -> ``ReplicaRouter`` spawns a leader + follower lockstep group (parallel/lockstep.py); the
test box has one GPU, so both ranks share it (gloo for the group, the one-shot IPC all-reduce for the
decode collectives).  Answers match the single-GPU TP=1 engine."""
import pytest
import torch

from llm_based_apache_spark_optimization_amd import prompts
from llm_based_apache_spark_optimization_amd.config import Settings

pytestmark = pytest.mark.gpu

SCHEMA = "Name (string)\nAge (int)\nCity (string)"
QUESTIONS = ["Select all records", "How many rows are there?", "Average age by city", "Oldest person"]


def test_tp2_replica_behind_fastapi(gpu, tmp_path):
    from fastapi.testclient import TestClient

    from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine
    from llm_based_apache_spark_optimization_amd.serving.fastapi_app import create_app
    from llm_based_apache_spark_optimization_amd.serving.service import make_context

    ref = build_engine("tiny-nsql", device=str(gpu), max_slots=4, max_model_len=512)
    want = [ref.generate([q], SamplingParams(max_tokens=8, ignore_eos=True), system=prompts.nl2sql_system(SCHEMA))[0].text
            for q in QUESTIONS]
    del ref
    torch.cuda.empty_cache()

    s = Settings(input_dir=str(tmp_path / "in"), output_dir=str(tmp_path / "out"),
                 history_dsn="sqlite:///" + str(tmp_path / "h.db"), engine="hip", tp=2, dp=1,
                 nl2sql_model="tiny-nsql", explain_model="tiny-llama3", max_batch=4, max_model_len=512,
                 kv_memory_fraction=0.05, secret_key="t", request_timeout_s=240)
    ctx = make_context(s)  # one visible GPU: the router maps both ranks of the replica onto it
    try:
        router = ctx.backend
        assert router.tp == 2 and len(router.replicas) == 1 and len(router.replicas[0].followers) == 1
        api = TestClient(create_app(ctx))
        got = []
        for q in QUESTIONS:
            r = api.post("/nl2sql", json={"question": q, "table_schema": SCHEMA,
                                          "options": {"num_predict": 8, "ignore_eos": True}})
            assert r.status_code == 200, r.text
            d = r.json()
            assert d["eval_count"] == 8
            got.append(d["sql_query"])
        # bf16 shards sum in a different order than the TP=1 GEMMs, so a near-tied greedy argmax of the random-init
        # model may flip in one answer; the sharded math itself is pinned at logit level (KL < 1e-6 against the
        # unsharded fp32 oracle) by tests/test_engine_cpu.py::test_tensor_parallel_matches_single
        assert sum(a == b for a, b in zip(got, want)) >= len(QUESTIONS) - 1, (got, want)
        assert router.health()["ok"]
    finally:
        ctx.backend.close(drain_s=5)

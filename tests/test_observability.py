"""Serving robustness and observability, CPU only:

* /metrics exports TTFT / TPOT / decode-rate histograms per model and route, engine span stages
  (queue / prefill / decode / detok), engine gauges, and per-replica load under the DP router;
* a failing engine step fails its requests at once and the loop keeps serving (restart);
* a fatal (device) error ends the loop; the service rebuilds the engine, and once the rebuild budget is
  spent the API answers 503 immediately instead of waiting for the request timeout.
"""
import time

import pytest
from fastapi.testclient import TestClient

from llm_based_apache_spark_optimization_amd.client import EngineService, EngineUnavailable
from llm_based_apache_spark_optimization_amd.config import Settings
from llm_based_apache_spark_optimization_amd.engine import build_engine
from llm_based_apache_spark_optimization_amd.serving.fastapi_app import create_app
from llm_based_apache_spark_optimization_amd.serving.service import make_context
from llm_based_apache_spark_optimization_amd.utils.metrics import REGISTRY

SCHEMA = "Name (string)\nAge (int)"


def _settings(tmp_path, **kw):
    return Settings(input_dir=str(tmp_path / "in"), output_dir=str(tmp_path / "out"),
                    history_dsn="sqlite:///" + str(tmp_path / "h.db"), engine="fake", nl2sql_model="tiny-nsql",
                    explain_model="tiny-llama3", secret_key="t", request_timeout_s=60, **kw)


def _service(builds):
    def factory(model):
        builds.append(model)
        return build_engine(model, device="cpu", max_slots=2, max_model_len=1024)

    return EngineService(factory, timeout_s=60, max_rebuilds=1)


def test_metrics_export_generation_histograms_and_engine_spans(tmp_path):
    builds = []
    svc = _service(builds)
    api = TestClient(create_app(make_context(_settings(tmp_path), backend=svc)))
    r = api.post("/nl2sql", json={"question": "Select all", "table_schema": SCHEMA,
                                  "options": {"num_predict": 6, "ignore_eos": True}})
    assert r.status_code == 200, r.text
    assert r.json()["eval_count"] == 6
    text = api.get("/metrics").text
    for needle in ('lsa_ttft_seconds_bucket{model="tiny-nsql",route="nl2sql"',
                   'lsa_tpot_seconds_count{model="tiny-nsql",route="nl2sql"} ',
                   'lsa_decode_tokens_per_second_bucket{model="tiny-nsql"',
                   'lsa_generated_tokens_total{model="tiny-nsql",route="nl2sql"}',
                   'lsa_stage_seconds_count{model="tiny-nsql",stage="engine_queue"}',
                   'lsa_stage_seconds_count{model="tiny-nsql",stage="engine_prefill"}',
                   'lsa_stage_seconds_count{model="tiny-nsql",stage="engine_decode"}',
                   'lsa_stage_seconds_count{model="tiny-nsql",stage="engine_detok"}',
                   'lsa_engine_running{model="tiny-nsql"}', 'lsa_engine_alive{model="tiny-nsql"} 1.0'):
        assert needle in text, needle
    assert REGISTRY.quantile("lsa_tpot_seconds", 0.5, model="tiny-nsql", route="nl2sql") > 0
    # the Ollama route is metered too
    r = api.post("/api/generate", json={"model": "tiny-nsql", "prompt": "x", "options": {"num_predict": 3}})
    assert r.status_code == 200
    assert 'lsa_ttft_seconds_count{model="tiny-nsql",route="api_generate"}' in api.get("/metrics").text


def test_failed_step_fails_requests_fast_and_loop_restarts(tmp_path):
    builds = []
    svc = _service(builds)
    svc.generate("tiny-nsql", "warm", options={"num_predict": 2})  # engine built and serving
    lp = svc.loop("tiny-nsql")
    real_step = lp.engine.step
    calls = {"n": 0}

    def flaky():
        calls["n"] += 1
        if calls["n"] == 1:
            raise ValueError("injected step failure")
        return real_step()

    lp.engine.step = flaky
    t0 = time.perf_counter()
    with pytest.raises(RuntimeError, match="injected step failure"):
        svc.generate("tiny-nsql", "a", options={"num_predict": 4})
    assert time.perf_counter() - t0 < 30  # released at once, not at the 60 s timeout
    assert lp.alive() and lp.restarts == 1
    assert lp.engine.sched.num_running == 0 and lp.engine.sched.num_waiting == 0  # slots / KV returned
    r = svc.generate("tiny-nsql", "b", options={"num_predict": 4, "ignore_eos": True})
    assert r.eval_count == 4
    h = svc.health()
    assert h["ok"] and h["engines"]["tiny-nsql"]["restarts"] == 1 and h["engines"]["tiny-nsql"]["aborted"] == 1
    assert builds == ["tiny-nsql"]  # recovered in place, no rebuild


def test_fatal_error_rebuilds_then_503(tmp_path):
    builds = []
    svc = _service(builds)
    api = TestClient(create_app(make_context(_settings(tmp_path), backend=svc)), raise_server_exceptions=False)

    def poison(lp):
        def boom():
            raise RuntimeError("HIP error: an illegal memory access was encountered")
        lp.engine.step = boom

    body = {"question": "q", "table_schema": SCHEMA, "options": {"num_predict": 3, "ignore_eos": True}}
    assert api.post("/nl2sql", json=body).status_code == 200
    poison(svc.loop("tiny-nsql"))
    r = api.post("/nl2sql", json=body)
    assert r.status_code == 500  # the request in flight when the device faulted fails
    assert not svc._loops["tiny-nsql"].alive()
    # next request: the dead engine is rebuilt (rebuild budget 1) and serves
    assert api.post("/nl2sql", json=body).status_code == 200
    assert builds == ["tiny-nsql", "tiny-nsql"] and svc.rebuilds["tiny-nsql"] == 1
    poison(svc.loop("tiny-nsql"))
    assert api.post("/nl2sql", json=body).status_code == 500
    t0 = time.perf_counter()
    r = api.post("/nl2sql", json=body)
    assert r.status_code == 503 and r.json()["error"] == "engine unavailable"
    assert time.perf_counter() - t0 < 5
    with pytest.raises(EngineUnavailable):
        svc.generate("tiny-nsql", "x")
    assert api.get("/ready").status_code == 503
    assert 'lsa_engine_alive{model="tiny-nsql"} 0.0' in api.get("/metrics").text


def test_router_metrics_per_replica_load(tmp_path):
    from llm_based_apache_spark_optimization_amd.parallel.router import ReplicaRouter

    router = ReplicaRouter(2, kind="fake", heartbeat_s=0.2, dead_after_s=10.0, timeout_s=60)
    try:
        t0 = time.time()
        while not all(r.ready for r in router.replicas) and time.time() - t0 < 60:
            time.sleep(0.05)
        api = TestClient(create_app(make_context(_settings(tmp_path), backend=router)))
        for _ in range(4):
            assert api.post("/nl2sql", json={"question": "q", "table_schema": SCHEMA}).status_code == 200
        h = router.health(deep=True)
        assert all(r.get("health", {}).get("ok") for r in h["replicas"])
        text = api.get("/metrics").text
        assert 'lsa_replica_alive{replica="0"} 1.0' in text and 'lsa_replica_alive{replica="1"} 1.0' in text
        served = [float(line.split()[-1]) for line in text.splitlines() if line.startswith("lsa_replica_served{")]
        assert sum(served) == 4 and min(served) >= 1  # least-outstanding dispatch used both replicas
        assert 'lsa_replica_inflight{replica="0"} 0' in text
    finally:
        router.close(drain_s=2)

"""Data-parallel replica router with fake replicas in subprocesses (CPU): dispatch fairness,
replica failure detection + re-dispatch, draining."""
import threading
import time

import pytest

from llm_based_apache_spark_optimization_amd.parallel.router import ReplicaRouter


@pytest.fixture
def router():
    r = ReplicaRouter(3, kind="fake", heartbeat_s=0.2, dead_after_s=5.0, timeout_s=60)
    yield r
    r.close(drain_s=2)


def test_dispatch_balances_load(router):
    out = []

    def go(i):
        out.append(router.generate("duckdb-nsql", f"q{i}", "s", {"fake_delay": 0.3}).response)

    ts = [threading.Thread(target=go, args=(i,)) for i in range(9)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert len(out) == 9 and all(o.startswith("SELECT") for o in out)
    served = [r["served"] for r in router.health()["replicas"]]
    assert sum(served) == 9 and max(served) - min(served) <= 1


def test_replica_death_redispatches(router):
    out, errs = [], []

    def go(i):
        try:
            out.append(router.generate("llama3.2", "explain", "troubleshoot", {"fake_delay": 1.0}).response)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=go, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    time.sleep(0.4)
    router.replicas[0].proc.kill()
    [t.join() for t in ts]
    assert not errs and len(out) == 6
    h = router.health()
    assert h["ok"] and not h["replicas"][0]["alive"]


def test_all_dead_raises():
    r = ReplicaRouter(1, kind="fake", heartbeat_s=0.2, timeout_s=10)
    try:
        r.generate("m", "warm")
        r.replicas[0].proc.kill()
        time.sleep(1.0)
        with pytest.raises(RuntimeError):
            r.generate("m", "x")
    finally:
        r.close(drain_s=0.5)


def test_streaming_through_router(router):
    whole = router.generate("duckdb-nsql", "q", "s").response
    chunks = list(router.generate_stream("duckdb-nsql", "q", "s"))
    assert chunks[-1].done and chunks[-1].response == "" and all(not c.done for c in chunks[:-1])
    assert "".join(c.response for c in chunks) == whole


def test_streaming_survives_replica_death(router):
    out = []

    def go():
        out.append("".join(c.response for c in router.generate_stream("llama3.2", "explain", "troubleshoot",
                                                                       {"fake_delay": 1.0})))

    ts = [threading.Thread(target=go) for _ in range(3)]
    [t.start() for t in ts]
    time.sleep(0.4)
    router.replicas[0].proc.kill()
    [t.join() for t in ts]
    expect = router.generate("llama3.2", "explain", "troubleshoot").response
    assert out == [expect] * 3


def _settings_kw(tmp_path, **over):
    import dataclasses

    from llm_based_apache_spark_optimization_amd.config import Settings

    s = Settings(input_dir=str(tmp_path / "in"), output_dir=str(tmp_path / "out"), engine="hip",
                 nl2sql_model="tiny-nsql", explain_model="tiny-llama3", max_batch=4, max_model_len=256,
                 secret_key="t", **over)
    return {f.name: getattr(s, f.name) for f in dataclasses.fields(s)}


def test_tp_replicas_serve_through_router(tmp_path):
    """dp=2 x tp=2 on CPU/gloo: each replica is a leader + follower lockstep TP group; answers match the
    single-process TP=1 engine (fp32 reduction order across shards may flip a late token, so the
    comparison is per prompt with a tolerance of one prompt), and both replicas answer identically."""
    from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine

    prompts = ["Select all records", "How many rows are there?", "total fare by vendor", "average age"]
    opts = {"num_predict": 8, "ignore_eos": True}
    ref = build_engine("tiny-nsql", device="cpu", max_slots=4, max_model_len=256)
    want = [ref.generate([p], SamplingParams(max_tokens=8, ignore_eos=True), system="T (int)")[0].text
            for p in prompts]
    r = ReplicaRouter(2, kind="hip", devices=[["", ""], ["", ""]], settings_kw=_settings_kw(tmp_path),
                      heartbeat_s=0.5, dead_after_s=120, timeout_s=240, tp=2)
    try:
        assert all(len(x.followers) == 1 for x in r.replicas)
        got = [None] * (2 * len(prompts))

        def go(i):
            got[i] = r.generate("tiny-nsql", prompts[i % len(prompts)], "T (int)", opts)

        ts = [threading.Thread(target=go, args=(i,)) for i in range(len(got))]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert all(g.eval_count == 8 for g in got)
        texts = [g.response for g in got]
        assert texts[: len(prompts)] == texts[len(prompts):]  # same prompt -> same answer on any replica
        assert sum(a == b for a, b in zip(texts, want)) >= len(prompts) - 1, (texts, want)
        served = [x["served"] for x in r.health()["replicas"]]
        assert min(served) >= 1  # both TP groups took requests
    finally:
        r.close(drain_s=5)
    for x in r.replicas:
        for p in [x.proc, *x.followers]:
            assert not p.is_alive()

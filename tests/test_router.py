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

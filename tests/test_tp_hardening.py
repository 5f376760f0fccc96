"""Failure handling of tensor-parallel replicas, on CPU (gloo, 2 processes):

* the IPC all-reduce set-up is collective and all-or-nothing: one rank failing to map its peers' regions makes
  every rank fall back to RCCL instead of the replica dying in ``TPGroup.warmup`` (parallel/custom_ar.py);
* TP ranks agree on one KV-arena size, so no rank owns fewer blocks than the leader's scheduler hands out;
* a lockstep follower whose replayed call raises leaves (exit code), and the leader's engine loop treats
  every step failure as fatal and runs its exit hook before releasing any caller (client._EngineLoop).
"""
import os
import queue
import socket
import threading
import time

import pytest
import torch


def _port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


class _FakeExt:
    """Stand-in for the HIP extension's region calls: allocations are integers, handles are bytes."""

    def __init__(self, rank: int):
        self.rank, self.freed, self.closed, self.next = rank, [], [], 1000 * (rank + 1)

    def ar_alloc(self, n):
        self.next += 1
        return self.next

    def ar_handle(self, p):
        return f"h{self.rank}:{p}".encode()

    def ar_open(self, h):
        self.next += 1
        return self.next

    def ar_close(self, p):
        self.closed.append(p)

    def ar_free(self, p):
        self.freed.append(p)


def _regions_worker(rank, world, port, fail_rank, q):
    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.parallel.custom_ar import IpcUnavailable, open_regions

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fail_rank is not None:
        os.environ["LSA_TEST_FAIL_AR_OPEN"] = str(fail_rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ext = _FakeExt(rank)
    try:
        base, ptrs, opened = open_regions(dist.group.WORLD, rank, world, ext, 4096)
        q.put((rank, "ok", len(ptrs), len(opened), ext.freed, ext.closed))
    except IpcUnavailable as e:
        q.put((rank, "unavailable", str(e), 0, ext.freed, ext.closed))
    dist.barrier()
    dist.destroy_process_group()


def _collect(ps, q, n, limit=60):
    got, t0 = {}, time.time()
    try:
        while len(got) < n:
            assert time.time() - t0 < limit, "workers timed out"
            assert not any(p.exitcode not in (None, 0) for p in ps), [p.exitcode for p in ps]
            try:
                r = q.get(timeout=1)
                got[r[0]] = r[1:]
            except queue.Empty:
                pass
    finally:
        [p.join(timeout=20) for p in ps]
        [p.kill() for p in ps if p.is_alive()]
    return got


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_ipc_region_setup_is_collective(fail_rank):
    import torch.multiprocessing as tmp

    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_regions_worker, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    [p.start() for p in ps]
    got = _collect(ps, q, 2)
    if fail_rank is None:
        assert all(v[0] == "ok" and v[1] == 2 and v[2] == 1 for v in got.values()), got
    else:
        # BOTH ranks give up (rank 0 mapped its peer fine) and release everything they made
        assert all(v[0] == "unavailable" for v in got.values()), got
        assert "rank 1" in got[0][1] and "injected" in got[0][1]
        assert all(len(v[3]) == 1 for v in got.values())  # own region freed on every rank
        assert len(got[0][4]) == 1  # rank 0 closed the peer region it had opened


def _min_worker(rank, world, port, q):
    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.engine.runner import ModelRunner
    from llm_based_apache_spark_optimization_amd.models import get_spec
    from llm_based_apache_spark_optimization_amd.models.llama import init_random
    from llm_based_apache_spark_optimization_amd.parallel import TPGroup

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPGroup(dist.group.WORLD, rank, world, torch.device("cpu"))
    w = init_random(get_spec("tiny-nsql"), "cpu", seed=0, tp_rank=rank, tp_size=world)
    # ranks that sized their arenas differently (own free memory): the runner takes the group's minimum
    r = ModelRunner(w, max_slots=2, max_model_len=256, tp=tp, num_kv_blocks=40 + 7 * rank)
    q.put((rank, r.num_kv_blocks, int(r.kv.shape[2])))
    dist.barrier()
    dist.destroy_process_group()


def test_tp_ranks_agree_on_kv_blocks():
    import torch.multiprocessing as tmp

    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_min_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    got = _collect(ps, q, 2, limit=120)
    assert got[0] == got[1] == (40, 40), got


class _BoomRunner:
    def decode(self, *a, **k):
        raise RuntimeError("boom")


class _Eng:
    runner = _BoomRunner()


def test_follower_leaves_when_a_replayed_call_raises():
    from multiprocessing import Pipe

    from llm_based_apache_spark_optimization_amd.parallel import lockstep

    a, b = Pipe()
    a.send(("build", "m"))
    a.send(("call", "m", "decode", (1, 2), {}))
    with pytest.raises(RuntimeError, match="boom"):  # exit_on_error=False: the error surfaces instead of _exit
        lockstep.follow(b, lambda m: _Eng(), exit_on_error=False)


class _StepFails:
    """Minimal engine: the first step raises; abort_all records that callers were released."""

    name = "m"

    def __init__(self):
        self.runner = None
        self.aborted = threading.Event()
        self.steps = 0

    def has_work(self):
        return self.steps == 0

    def step(self):
        self.steps += 1
        raise RuntimeError("step failed after a mirrored call")

    def abort_all(self, reason):
        self.aborted.set()
        return []


def test_tp_leader_loop_treats_every_step_error_as_fatal():
    from llm_based_apache_spark_optimization_amd.client import _EngineLoop

    seen = []
    eng = _StepFails()
    lp = _EngineLoop(eng, every_error_fatal=True, on_fatal=lambda e: seen.append((repr(e), eng.aborted.is_set())))
    lp._t.join(timeout=10)
    assert not lp.alive() and eng.steps == 1
    assert seen and "mirrored" in seen[0][0] and seen[0][1] is False  # the hook ran before callers were released
    # without the TP flag the same error is survivable: the loop aborts the requests and keeps serving
    eng2 = _StepFails()
    lp2 = _EngineLoop(eng2)
    assert eng2.aborted.wait(10)
    time.sleep(0.2)
    assert lp2.alive()
    lp2.close()

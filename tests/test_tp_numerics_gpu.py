"""TP=2 decode logits with the bf16 IPC all-reduce payload (the default since round 5, parallel/custom_ar.py) against
the fp32 oracle on the unsharded weights and against the TP=1 engine (TP parity of the bf16 default).
Two processes: each rank on its own GPU when the box has two, else both on the one GPU (gloo for the group, the
one-shot IPC all-reduce for the decode collectives, as in tests/test_tp_launches_gpu.py).  Both ranks run the same
teacher-forced decode (SPMD); rank 0 compares."""
import queue
import socket
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

PROMPTS = [[1] + list(range(5, 90)), [1, 7, 7, 9, 11]]
STEPS = 16


def _worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.engine import build_engine
    from llm_based_apache_spark_optimization_amd.eval import numerics as nm
    from llm_based_apache_spark_optimization_amd.parallel import TPGroup

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", rank if torch.cuda.device_count() >= world else 0)
    torch.cuda.set_device(dev)
    out = {}
    try:
        tpg = TPGroup(dist.group.WORLD, rank, world, dev)
        e = build_engine("tiny-nsql", device=str(dev), max_slots=4, max_model_len=256, tp=tpg, seed=3)
        toks, elog = nm.record_decode_logits(e, PROMPTS, STEPS)
        out["describe"] = tpg.describe()
        out["toks"] = toks
        if rank == 0:
            full = build_engine("tiny-nsql", device=str(dev), max_slots=4, max_model_len=256, seed=3)
            out["oracle"] = nm.check_recorded(e, PROMPTS, toks, elog, STEPS, check_rows=(0, 1), weights=full.runner.w)
            # the TP=1 engine teacher-forced on the TP=2 tokens: logit-level KL between the two engines
            t1, l1 = nm.record_decode_logits(full, PROMPTS, STEPS)
            kl = [nm.compare(l1[i], elog[i])["kl"] for i in range(len(PROMPTS)) if t1[i] == toks[i]]
            out["same_tokens"] = [t1[i] == toks[i] for i in range(len(PROMPTS))]
            out["kl_tp1_tp2_max"] = float(torch.cat(kl).max()) if kl else None
    except Exception as ex:  # noqa: BLE001
        out["error"] = repr(ex)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_tp2_bf16_allreduce_logits_match_oracle_and_tp1(gpu):
    import torch.multiprocessing as tmp

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = tmp.get_context("spawn")
    qu = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, qu)) for r in range(2)]
    [p.start() for p in ps]
    got, t0 = {}, time.time()
    try:
        while len(got) < 2:
            assert time.time() - t0 < 180, "TP workers timed out"
            assert not any(p.exitcode not in (None, 0) for p in ps), [p.exitcode for p in ps]
            try:
                r, res = qu.get(timeout=2)
                got[r] = res
            except queue.Empty:
                pass
    finally:
        [p.join(timeout=30) for p in ps]
    for r in range(2):
        assert "error" not in got[r], got[r]
    d = got[0]["describe"]
    assert d["ipc_allreduce"] and d["ipc_bf16_payload"], d  # the default under test: bf16 payloads on the IPC kernel
    assert got[0]["toks"] == got[1]["toks"]  # every rank decodes the same tokens
    num = got[0]["oracle"]
    assert num["class"] == "bf16" and num["ok"], num  # the bf16 numerics class, unchanged by the bf16 partials
    # where both engines chose the same tokens, their logits agree to bf16-rounding level at every step
    if got[0]["kl_tp1_tp2_max"] is not None:
        assert got[0]["kl_tp1_tp2_max"] < 1e-2, got[0]
    assert any(got[0]["same_tokens"]), got[0]

"""A TP=2 decode step issues no more launches per layer than TP=1: the row-parallel
projections' residual add, bf16 / fragment-major activations and row sums ride in the one-shot IPC all-reduce
(csrc/kernels/allreduce.hip RES epilogue), so each layer is  ar_res | qkv | attention | o | ar_res | gate_up | down.
Kernel launches are counted on the captured decode graph (hipGraphGetNodes).  Two processes share the test box's
one GPU (gloo exchanges the IPC handles); on the 8-GPU node the same kernels run over xGMI."""
import queue
import socket
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

LAYERS = 4


def _build(tp_group, dev):
    import dataclasses

    from llm_based_apache_spark_optimization_amd.engine import ModelRunner
    from llm_based_apache_spark_optimization_amd.models import get_spec
    from llm_based_apache_spark_optimization_amd.models.llama import init_random

    spec = dataclasses.replace(get_spec("tiny-nsql"), n_layers=LAYERS)
    tpr, tps = (tp_group.rank, tp_group.size) if tp_group is not None else (0, 1)
    w = init_random(spec, dev, seed=1, tp_rank=tpr, tp_size=tps)
    return ModelRunner(w, max_slots=32, max_model_len=512, tp=tp_group, num_kv_blocks=32 * 8 + 1)


def _worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.parallel import TPGroup

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", rank if torch.cuda.device_count() >= world else 0)  # own GPU when there are enough
    torch.cuda.set_device(dev)
    out = {}
    try:
        tpg = TPGroup(dist.group.WORLD, rank, world, dev)
        r = _build(tpg, dev)
        out["fused"] = r.tp.car is not None
        out["n32"] = r.count_step_kernels(32)
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_tp2_step_launches_no_more_than_tp1(gpu):
    import torch.multiprocessing as tmp

    tp1 = _build(None, gpu).count_step_kernels(32)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    got, t0 = {}, time.time()
    try:
        while len(got) < 2:
            assert time.time() - t0 < 150, "TP workers timed out"
            assert not any(p.exitcode not in (None, 0) for p in ps), [p.exitcode for p in ps]
            try:
                r, res = q.get(timeout=2)
                got[r] = res
            except queue.Empty:
                pass
    finally:
        [p.join(timeout=30) for p in ps]
    for r in range(2):
        assert "error" not in got[r], got[r]
        assert got[r]["fused"], "the one-shot IPC all-reduce must be available between the test ranks"
    tp2 = got[0]["n32"]
    print({"tp1_kernels": tp1, "tp2_kernels": tp2, "layers": LAYERS})
    # once per step TP adds three launches: the last down projection's all-reduce ahead of the final RMSNorm (TP = 1
    # sums its slabs inside that launch), the vocab-parallel logits' one-shot all-gather and its rank-major ->
    # row-major copy (measured 32 -> 35 at 4 layers); any extra launch per layer would add LAYERS = 4 more
    assert tp2 <= tp1 + 3 < tp1 + LAYERS, (tp1, tp2)

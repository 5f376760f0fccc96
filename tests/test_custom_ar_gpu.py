"""IPC all-reduce kernels (csrc/kernels/allreduce.hip): one-shot and two-shot (reduce-scatter +
all-gather), f32 and bf16 payloads, vs the fp32 rank-ordered sum of the same (rounded) contributions.  Rank r runs on
cuda:r when the box has at least `world` GPUs (peer regions mapped across devices over xGMI), else every rank shares
cuda:0 (IPC handles of the same device).  gloo exchanges the handles."""
import queue
import socket
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [4, 4096, 32 * 4096, 64 * 4096 + 4]  # B=1 .. B=64 decode rows of d=4096, plus a ragged tail


def _inputs(rank: int, it: int, n: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 * it + 17 * rank + n)
    return torch.randn(n, generator=g)


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).float()


# kernel variants: (bf16 payload, two-shot) -- the reference rounds each rank's contribution as the kernel does
VARIANT = (False, False)


def _expected(world: int, it: int, n: int, variant=None) -> torch.Tensor:
    bf16, two = VARIANT if variant is None else variant
    acc = torch.zeros(n)
    for r in range(world):  # the kernel's summation order
        x = _inputs(r, it, n)
        acc = acc + (_bf(x) if bf16 else x)
    return _bf(acc) if (bf16 and two) else acc  # the two-shot owner pushes the bf16 sum


def _device(rank: int, world: int) -> torch.device:
    """cuda:rank when every rank has a GPU of its own (the cross-device IPC path), else the shared cuda:0."""
    return torch.device("cuda", rank if torch.cuda.device_count() >= world else 0)


def _worker(rank, world, port, q, variant=(False, False)):
    global VARIANT
    VARIANT = variant
    import os

    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.parallel.custom_ar import IpcAllReduce

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = _device(rank, world)
    torch.cuda.set_device(dev)
    errs = []
    bf16, two = variant
    try:
        car = IpcAllReduce(dist.group.WORLD, rank, world, dev, max_bytes=4 << 20, timeout_s=30, bf16=bf16,
                           two_shot_min_bytes=0 if two else 1 << 40)
        assert car.mode(4096) == (1 if bf16 else 0) | (2 if (two and world > 2) else 0) or (two and world == 2)
        if two and world == 2:
            car.two_shot_min_bytes = -1
            car.mode = lambda nbytes: (1 if bf16 else 0) | 2  # exercise the two-shot kernel at TP = 2 too
        it = 0
        for n in SIZES:  # eager, several epochs per size (both slot parities, block counts change)
            for _ in range(3):
                t = _inputs(rank, it, n).to(dev)
                car(t)
                if not torch.equal(t.cpu(), _expected(world, it, n)):
                    errs.append(f"eager n={n} it={it}: max err {(t.cpu() - _expected(world, it, n)).abs().max()}")
                # stated bound vs the exact sum: each bf16 rounding (RNE, 8 significant bits) moves a value by <= 2^-8 of it
                xs = [_inputs(r, it, n) for r in range(world)]
                exact = torch.stack(xs).double().sum(0)
                # (plus the f32 rank-ordered summation: <= world * 2^-24 of the sum of magnitudes)
                mag = torch.stack(xs).abs().double().sum(0)
                bound = mag * (2.0 ** -8 * bf16 + world * 2.0 ** -24) + exact.abs() * 2.0 ** -8 * (bf16 and two) + 1e-30
                if ((t.cpu().double() - exact).abs() > bound).any():
                    errs.append(f"bound n={n} it={it}")
                it += 1
        for ns, n in ((2, 4096), (4, 32 * 4096), (3, 4100)):  # split-K slabs folded into the all-reduce
            slabs = [_inputs(rank, it + 100 * k, n) for k in range(ns)]
            t = torch.stack(slabs).to(dev)
            red = car.reduce_slabs(t)
            want = torch.zeros(n)
            for r in range(world):
                own = _inputs(r, it, n)
                for k in range(1, ns):
                    own = own + _inputs(r, it + 100 * k, n)
                want = want + (_bf(own) if bf16 else own)
            if bf16 and two:
                want = _bf(want)
            if red.shape[0] != 1 or not torch.equal(red[0].cpu(), want):
                errs.append(f"slabs ns={ns} n={n} it={it}")
            it += 1
        # residual epilogue fused into the all-reduce (TPGroup.reduce_add): h += sum over ranks of each rank's slab
        # sum, xn = bf16(h) (row-major and fragment-major), ss += row sums of h^2 in Q24 -- against fp32 PyTorch
        from llm_based_apache_spark_optimization_amd import ops

        for ns, rows, D in ((2, 1, 3072), (4, 32, 4096), (1, 20, 4096)):
            n = rows * D
            slabs = torch.stack([_inputs(rank, it + 100 * k, n) for k in range(ns)]).view(ns, rows, D).to(dev)
            h0 = _inputs(7, it, n).view(rows, D)
            h = h0.to(dev).clone()
            xmt = ops.xfrag_tiles(rows) if rows > 16 else 0
            xn = torch.zeros((xmt * 16 if xmt else rows) * D, dtype=torch.bfloat16, device=dev)
            ss = torch.full((rows,), 5, dtype=torch.int64, device=dev)
            car.reduce_slabs_res(slabs, h, xn, ss, xmt)
            tot = torch.zeros(rows, D)
            for r in range(world):
                own = sum(_inputs(r, it + 100 * k, n) for k in range(ns)).view(rows, D)
                tot = tot + (_bf(own) if bf16 else own)
            if bf16 and two:
                tot = _bf(tot)
            want = h0 + tot
            if (h.cpu() - want).abs().max() > 1e-4 * want.abs().max():
                errs.append(f"res h ns={ns} rows={rows}")
            xr = ops.from_xfrag(xn, rows, D) if xmt else xn.view(rows, D)
            if not torch.equal(xr.cpu(), h.cpu().to(torch.bfloat16)):
                errs.append(f"res xn rows={rows} xmt={xmt}")
            ssw = (ss.cpu() - 5).double() / ops.SS_SCALE
            if not torch.allclose(ssw, h.cpu().double().pow(2).sum(1), rtol=1e-5):
                errs.append(f"res ss rows={rows}")
            it += 1
        for n in (4096, 32 * 16000):  # all-gather (vocab-parallel logits), rank-major output
            t = _inputs(rank, it, n).to(dev)
            out = torch.empty(world * n, device=dev)
            car.all_gather(out, t)
            want = torch.cat([_inputs(r, it, n) for r in range(world)])
            if not torch.equal(out.cpu(), want):
                errs.append(f"gather n={n} it={it}")
            it += 1
        # captured in a hipGraph, replayed with new inputs copied into the captured buffer
        n = 32 * 4096
        buf = torch.zeros(n, device=dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                car(buf)
        torch.cuda.current_stream(dev).wait_stream(s)
        dist.barrier()
        for _ in range(5):
            buf.copy_(_inputs(rank, it, n).to(dev))
            g.replay()
            if not torch.equal(buf.cpu(), _expected(world, it, n)):
                errs.append(f"graph it={it}")
            it += 1
        torch.cuda.synchronize(dev)
        car.check()
        car.close()
    except Exception as e:  # noqa: BLE001
        errs.append(repr(e))
    q.put((rank, errs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("variant", [(False, False), (True, False), (False, True), (True, True)],
                         ids=["f32_oneshot", "bf16_oneshot", "f32_twoshot", "bf16_twoshot"])
def test_ipc_allreduce_matches_rank_ordered_sum(gpu, world, variant):
    """Every kernel variant equals the rank-ordered f32 sum of the contributions as pushed (bf16: each rounded to
    bf16; two-shot bf16: the sum rounded too), bitwise on every rank; and the bf16 variants stay within the bf16
    rounding bound of the exact fp32 sum: |result - sum| <= 2^-9 (sum of |x_r|, + |sum| for the two-shot bf16
    sum) + 1e-6 |sum|."""
    import torch.multiprocessing as tmp

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, variant)) for r in range(world)]
    [p.start() for p in ps]
    got, t0 = {}, time.time()
    try:
        while len(got) < world:
            assert time.time() - t0 < 100, "all-reduce workers timed out"
            assert not any(p.exitcode not in (None, 0) for p in ps), [p.exitcode for p in ps]
            try:
                r, errs = q.get(timeout=2)
                got[r] = errs
            except queue.Empty:
                pass
    finally:
        [p.join(timeout=30) for p in ps]
        [p.kill() for p in ps if p.is_alive()]
    assert all(not e for e in got.values()), got


def _engine_worker(rank, world, port, q):
    """TP=2 tiny engine; after one good generate, rank 1 stops participating (alive, idle) and rank 0's
    next generate must raise (the one-shot all-reduce times out, poisons its output and sets err)."""
    import datetime
    import os

    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine
    from llm_based_apache_spark_optimization_amd.engine.runner import TPCommError
    from llm_based_apache_spark_optimization_amd.parallel import TPGroup

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LSA_CUSTOM_AR_TIMEOUT_S="0.3")
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    dev = _device(rank, world)
    torch.cuda.set_device(dev)
    out = []
    try:
        tp = TPGroup(dist.group.WORLD, rank, world, dev)
        eng = build_engine("tiny-nsql", device=str(dev), max_slots=2, max_model_len=256, tp=tp)
        assert tp.car is not None
        sp = SamplingParams(max_tokens=4, ignore_eos=True)
        good = eng.generate([[1, 5, 6, 7, 8]], sp)[0].token_ids
        out.append(("good", good))
        dist.barrier()
        if rank == 0:
            try:
                eng.generate([[1, 5, 6, 7, 8]], sp)
                out.append(("no-error", None))
            except TPCommError as e:
                out.append(("raised", str(e)[:60]))
        else:
            time.sleep(8)  # alive but silent: rank 0's all-reduces find no peer
        torch.cuda.synchronize(dev)
    except Exception as e:  # noqa: BLE001
        out.append(("exc", repr(e)))
    q.put((rank, out))


def test_engine_ar_timeout_raises(gpu):
    import torch.multiprocessing as tmp

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    got, t0 = {}, time.time()
    try:
        while len(got) < 2:
            assert time.time() - t0 < 110, "engine workers timed out"
            assert not any(p.exitcode not in (None, 0) for p in ps), [p.exitcode for p in ps]
            try:
                r, out = q.get(timeout=2)
                got[r] = out
            except queue.Empty:
                pass
    finally:
        [p.join(timeout=30) for p in ps]
        [p.kill() for p in ps if p.is_alive()]
    assert got[0][0][0] == "good" and got[1][0][0] == "good" and got[0][0][1] == got[1][0][1], got
    assert got[0][1][0] == "raised", got


def _spawn(target, world, limit):
    import torch.multiprocessing as tmp

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    got, t0 = {}, time.time()
    try:
        while len(got) < world:
            assert time.time() - t0 < limit, "workers timed out"
            assert not any(p.exitcode not in (None, 0) for p in ps), [p.exitcode for p in ps]
            try:
                r, out = q.get(timeout=2)
                got[r] = out
            except queue.Empty:
                pass
    finally:
        [p.join(timeout=30) for p in ps]
        [p.kill() for p in ps if p.is_alive()]
    return got


def _follower_timeout_worker(rank, world, port, q):
    """Rank 1 (a follower) times out waiting for rank 0; rank 0's NEXT call must see the abort word rank 1
    raised in its region: poisoned (NaN) result and err set, so the leader's host sync raises."""
    import os

    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.parallel.custom_ar import IpcAllReduce

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = _device(rank, world)
    torch.cuda.set_device(dev)
    out = {}
    try:
        car = IpcAllReduce(dist.group.WORLD, rank, world, dev, max_bytes=1 << 20, timeout_s=0.5)
        t = torch.ones(4096, device=dev)
        car(t)
        torch.cuda.synchronize(dev)
        out["good"] = bool(torch.all(t == world).item())
        dist.barrier()
        if rank == 1:
            t = torch.ones(4096, device=dev)
            car(t)  # rank 0 is asleep: times out after 0.5 s
            torch.cuda.synchronize(dev)
            out["err"] = int(car.err.item())
            dist.barrier()
        else:
            dist.barrier()  # rank 1's call has timed out and raised the abort word
            t = torch.ones(4096, device=dev)
            car(t)  # rank 1's flag for this epoch is up: no wait, but the abort word is set
            torch.cuda.synchronize(dev)
            out["err"] = int(car.err.item())
            out["nan"] = bool(torch.isnan(t).all().item())
        dist.barrier()
    except Exception as e:  # noqa: BLE001
        out["exc"] = repr(e)
    q.put((rank, out))


def test_follower_timeout_poisons_the_leader(gpu):
    got = _spawn(_follower_timeout_worker, 2, 90)
    assert got[0].get("good") and got[1].get("good"), got
    assert got[1]["err"] == 1, got
    assert got[0]["err"] == 1 and got[0]["nan"], got


def _fallback_worker(rank, world, port, q):
    """TP=2 tiny engine with rank 1's peer mapping forced to fail: both ranks fall back to the plain
    collectives (no IPC all-reduce) and generate the same tokens as the IPC path."""
    import os

    import torch.distributed as dist

    from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine
    from llm_based_apache_spark_optimization_amd.parallel import TPGroup

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = _device(rank, world)
    torch.cuda.set_device(dev)
    out = {}
    try:
        sp = SamplingParams(max_tokens=12, ignore_eos=True)
        prompts = [[1, 5, 6, 7, 8], [1] + list(range(20, 90))]
        os.environ["LSA_TEST_FAIL_AR_OPEN"] = "1"
        tp = TPGroup(dist.group.WORLD, rank, world, dev)
        eng = build_engine("tiny-nsql", device=str(dev), max_slots=2, max_model_len=256, tp=tp)
        out["fallback_car"] = tp.car is None
        out["fallback"] = [r.token_ids for r in eng.generate(prompts, sp)]
        del eng
        os.environ.pop("LSA_TEST_FAIL_AR_OPEN")
        tp2 = TPGroup(dist.new_group([0, 1]), rank, world, dev)
        eng2 = build_engine("tiny-nsql", device=str(dev), max_slots=2, max_model_len=256, tp=tp2)
        out["ipc_car"] = tp2.car is not None
        out["ipc"] = [r.token_ids for r in eng2.generate(prompts, sp)]
        torch.cuda.synchronize(dev)
        dist.barrier()
    except Exception as e:  # noqa: BLE001
        out["exc"] = repr(e)
    q.put((rank, out))


def test_ar_open_failure_falls_back_with_identical_tokens(gpu):
    got = _spawn(_fallback_worker, 2, 150)
    for r in (0, 1):
        assert "exc" not in got[r], got
        assert got[r]["fallback_car"] and got[r]["ipc_car"], got
    assert got[0]["fallback"] == got[0]["ipc"] == got[1]["fallback"], got

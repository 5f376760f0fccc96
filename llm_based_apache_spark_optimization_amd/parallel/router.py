"""Data-parallel request dispatch over engine replica processes (SURVEY.md §2.6 P-DP).

The reference serves everything from one process with one global model handle (FastAPI/app.py:19,
Flask/app.py:16).  Here the front end (FastAPI / Flask / the eval harness) talks to a
``ReplicaRouter`` that owns ``dp`` worker processes, each pinned to its own GPU (or GPU group for a
TP replica) through ``HIP_VISIBLE_DEVICES`` set before the worker touches the GPU, each running its
own continuous-batching engines.  No GPU collective is needed in steady state: replicas are
independent and initialise identical random weights from the same seed (or load the same
checkpoint).

* dispatch: least outstanding requests (ties -> fewest dispatched, then lowest replica id);
* failure detection: a dead worker process (exit) or, once the replica has sent its first heartbeat
  (backends built), a missed heartbeat marks the replica down; its
  in-flight requests are re-dispatched to the remaining replicas (at-least-once; generation is
  idempotent for greedy decoding and seeded sampling);
* drain: ``close()`` stops accepting, waits for in-flight requests, then stops the workers;
* streaming: a worker forwards its backend's response pieces as they decode; after a re-dispatch the
  new replica's pieces are replayed from the start and the text already delivered is skipped.
"""
from __future__ import annotations

import itertools
import logging
import multiprocessing as mp
import os
import queue
import threading
import time
from typing import Iterator, Optional

from ..client import Backend, GenerateResponse

log = logging.getLogger(__name__)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_gpus() -> int:
    """GPU count without initialising HIP in this process (the router must not touch the GPU before
    its workers are spawned)."""
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if env:
        return len([x for x in env.split(",") if x.strip()])
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def _tp_local_device(tp_rank: int, shared_device: bool) -> int:
    """Index of this TP rank's GPU in its own view: every rank of a replica sees the replica's whole GPU
    list (as torchrun ranks do) and owns entry ``tp_rank``, so peers are visible devices and
    ``hipDeviceCanAccessPeer`` can be checked before the IPC all-reduce maps them; ranks sharing one GPU
    (test boxes) see only that GPU."""
    return 0 if shared_device else tp_rank


def _init_tp_rank(tp_rank: int, tp_size: int, port: int, shared_device: bool) -> None:
    """torch.distributed world = this replica's TP ranks (one process per GPU; RCCL when every rank
    owns its own GPU, gloo when ranks share one device (test boxes) or there is no GPU)."""
    import torch
    import torch.distributed as dist

    local = _tp_local_device(tp_rank, shared_device)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(tp_rank),
                      WORLD_SIZE=str(tp_size), LOCAL_RANK=str(local))
    if torch.cuda.is_available() and not shared_device:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        dist.init_process_group("gloo")


def _tp_engine_factory(settings, tp_rank: int, tp_size: int):
    """model -> LLMEngine holding this rank's shard; each model gets its own TP group (own RCCL
    communicator + IPC all-reduce region), created collectively inside the lockstep ``build``."""
    import torch
    import torch.distributed as dist

    from ..serving.service import engine_factory
    from .tp import TPGroup

    def tp_for_model():
        g = dist.new_group(list(range(tp_size)))
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        return TPGroup(g, tp_rank, tp_size, dev)

    return engine_factory(settings, tp_factory=tp_for_model)


def _worker(conn, replica: int, devices: str, kind: str, settings_kw: dict, heartbeat_s: float,
            tp_rank: int = 0, tp_size: int = 1, port: int = 0, peers=None, shared_device: bool = False):
    """Replica process: build backends lazily, answer requests until told to stop.

    TP replicas (tp_size > 1): rank 0 is the leader (``conn`` = router pipe, ``peers`` = pipes to its
    followers); ranks > 0 are followers (``conn`` = pipe from the leader) that mirror its runner calls
    (parallel/lockstep.py).  ``devices``: this process's HIP_VISIBLE_DEVICES -- a TP rank gets its
    replica's whole GPU list and selects entry ``tp_rank`` (``_tp_local_device``)."""
    if devices:
        os.environ["HIP_VISIBLE_DEVICES"] = devices  # before any HIP call in this process
    from ..config import Settings
    from ..client import EngineService, FakeBackend

    chan = None
    if tp_size > 1:
        from . import lockstep

        _init_tp_rank(tp_rank, tp_size, port, shared_device)
        s = Settings(**settings_kw)
        build = _tp_engine_factory(s, tp_rank, tp_size)
        if tp_rank > 0:
            lockstep.follow(conn, build)
            return
        chan = lockstep.LeaderChannel(peers or [])
        defaults = {"temperature": s.temperature, "top_k": s.top_k, "top_p": s.top_p, "num_predict": s.max_new_tokens}

        def die(e: BaseException) -> None:
            # any failed step leaves the lockstep group out of step (followers may sit in collectives the
            # leader never joins): never step it again -- exit, so the router re-dispatches the in-flight
            # requests to live replicas and terminates this replica's followers
            log.error("TP replica %d leader: engine step failed (%r); exiting", replica, e)
            os._exit(70)

        backend = EngineService(lockstep.lockstep_factory(build, chan), defaults=defaults,
                                timeout_s=s.request_timeout_s, max_rebuilds=0, every_error_fatal=True,
                                on_fatal=die)
    elif kind == "fake":
        backend = FakeBackend()
    else:
        from ..serving.service import backend_from_settings

        s = Settings(**settings_kw)
        s.dp, s.tp = 1, 1
        backend = backend_from_settings(s)
    lock = threading.Lock()

    def send(msg):
        with lock:
            conn.send(msg)

    def beat():
        while True:
            try:
                send(("hb", replica, time.time()))
            except (OSError, EOFError):
                return
            time.sleep(heartbeat_s)

    threading.Thread(target=beat, daemon=True).start()

    def serve(rid, model, prompt, system, options, raw=False, stream=False):
        if prompt == "__lsa_crash__":  # fault injection for tests
            os._exit(3)
        try:
            if stream:
                for c in backend.generate_stream(model, prompt, system, options, raw):
                    if not c.done:
                        send(("piece", rid, c.response))
                    else:
                        send(("ok", rid, c.to_dict()))
            else:
                r = backend.generate(model, prompt, system, options, raw)
                send(("ok", rid, r.to_dict()))
        except Exception as e:  # noqa: BLE001
            send(("err", rid, repr(e)))

    pool = []
    while True:
        try:
            msg = conn.recv()
        except (EOFError, OSError):
            msg = ("stop",)
        if msg[0] == "stop":
            if chan is not None:
                chan.close()  # followers leave their replay loops
            return
        if msg[0] == "gen":
            t = threading.Thread(target=serve, args=msg[1:], daemon=True)  # concurrency -> batching
            t.start()
            pool.append(t)
        elif msg[0] == "health":  # the router's deep health probe: this replica's engine gauges
            try:
                send(("health", msg[1], backend.health()))
            except Exception as e:  # noqa: BLE001
                send(("health", msg[1], {"ok": False, "error": repr(e)}))


class _Replica:
    def __init__(self, idx: int, proc, conn, followers=()):
        self.idx, self.proc, self.conn = idx, proc, conn
        self.followers = list(followers)  # TP ranks > 0 of this replica (no pipe to the router)
        self.inflight: dict = {}
        self.alive = True
        self.last_hb = time.time()
        self.ready = False  # first heartbeat seen: start-up (imports, weight load) is not a missed beat
        self.served = 0
        self.send_lock = threading.Lock()


class ReplicaRouter(Backend):
    def __init__(self, dp: int, kind: str = "hip", devices: Optional[list] = None, settings_kw: Optional[dict] = None,
                 heartbeat_s: float = 2.0, dead_after_s: float = 30.0, timeout_s: float = 300.0, tp: int = 1):
        """``devices[i]``: replica i's GPU ids, one per TP rank (comma-separated string or list); each
        rank process sees only its own GPU.  ``tp > 1``: every replica is a lockstep TP group."""
        self.kind = kind
        self.tp = max(1, int(tp))
        self.timeout_s = timeout_s
        self.dead_after_s = dead_after_s
        self._ids = itertools.count(1)
        self._lock = threading.Lock()
        self._waiters: dict = {}
        self._probes: dict = {}
        self._closing = False
        ctx = mp.get_context("spawn")
        self.replicas = []
        for i in range(dp):
            a, b = ctx.Pipe()
            if devices:
                dev = devices[i].split(",") if isinstance(devices[i], str) else [str(x) for x in devices[i]]
            else:
                dev = [str(i * self.tp + j) if kind != "fake" else "" for j in range(self.tp)]
            if self.tp == 1:
                p = ctx.Process(target=_worker, args=(b, i, ",".join(dev), kind, settings_kw or {}, heartbeat_s),
                                daemon=True)
                p.start()
                self.replicas.append(_Replica(i, p, a))
                continue
            # TP replica: rank 0 leads (router pipe + one pipe per follower), ranks > 0 follow
            assert len(dev) == self.tp, f"replica {i}: {len(dev)} devices for tp={self.tp}"
            port = _free_port()
            shared = len(set(dev)) < len(dev)  # ranks sharing one GPU (test boxes): gloo, not RCCL
            lead_ends, followers = [], []
            vis = (lambda j: dev[j]) if shared else (lambda j: ",".join(dev))
            for j in range(1, self.tp):
                lc, fc = ctx.Pipe()
                lead_ends.append(lc)
                fp = ctx.Process(target=_worker, args=(fc, i, vis(j), kind, settings_kw or {}, heartbeat_s, j,
                                                       self.tp, port, None, shared), daemon=True)
                fp.start()
                followers.append(fp)
            p = ctx.Process(target=_worker, args=(b, i, vis(0), kind, settings_kw or {}, heartbeat_s, 0, self.tp,
                                                  port, lead_ends, shared), daemon=True)
            p.start()
            self.replicas.append(_Replica(i, p, a, followers))
        for r in self.replicas:
            threading.Thread(target=self._reader, args=(r,), daemon=True).start()
        threading.Thread(target=self._monitor, daemon=True).start()

    @staticmethod
    def from_settings(settings) -> "ReplicaRouter":
        import dataclasses

        kw = {f.name: getattr(settings, f.name) for f in dataclasses.fields(settings)}
        tp, dp = max(1, settings.tp), max(1, settings.dp)
        kind = "fake" if settings.engine == "fake" else "hip"
        ngpu = _visible_gpus() if kind == "hip" else 0
        if kind == "hip" and ngpu and dp * tp > ngpu:
            log.warning("dp=%d x tp=%d needs %d GPUs, %d visible: ranks share GPUs (round-robin)", dp, tp, dp * tp, ngpu)
        env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
        ids = [x.strip() for x in env.split(",") if x.strip()] if env else [str(k) for k in range(ngpu)]
        devices = [[ids[(i * tp + j) % ngpu] if ngpu else "" for j in range(tp)] for i in range(dp)]
        return ReplicaRouter(dp, kind, devices, kw, timeout_s=settings.request_timeout_s, tp=tp)

    # ------------------------------------------------------------------------------ internals
    def _reader(self, r: _Replica):
        while True:
            try:
                msg = r.conn.recv()
            except (EOFError, OSError):
                self._mark_dead(r, "pipe closed")
                return
            if msg[0] == "hb":
                r.last_hb = time.time()
                r.ready = True
                continue
            kind, rid, payload = msg
            if kind == "health":
                with self._lock:
                    w = self._probes.get(rid)
                if w is not None:
                    w[1] = payload
                    w[0].set()
                continue
            if kind == "piece":
                with self._lock:
                    w = self._waiters.get(rid) if rid in r.inflight else None  # a stale replica's pieces drop
                if w is not None and w[2] is not None:
                    w[2].put(("piece", payload))
                continue
            with self._lock:
                r.inflight.pop(rid, None)
                r.served += 1
                w = self._waiters.get(rid)
            if w is not None:
                self._finish(w, (kind, payload))

    def _monitor(self):
        while not self._closing:
            time.sleep(0.5)
            for r in self.replicas:
                hb_lost = r.ready and time.time() - r.last_hb > self.dead_after_s
                procs_ok = r.proc.is_alive() and all(f.is_alive() for f in r.followers)
                if r.alive and (not procs_ok or hb_lost):
                    self._mark_dead(r, "process exited" if not procs_ok else "heartbeat lost")
                    for p in [r.proc, *r.followers]:  # a TP group missing a rank can never step again
                        if p.is_alive():
                            p.terminate()

    def _mark_dead(self, r: _Replica, why: str):
        with self._lock:
            if not r.alive:
                return
            r.alive = False
            orphans = list(r.inflight.items())
            r.inflight.clear()
        log.error("replica %d down (%s); re-dispatching %d request(s)", r.idx, why, len(orphans))
        for rid, req in orphans:
            w = self._waiters.get(rid)
            if w is not None and w[2] is not None:
                w[2].put(("restart", None))
            try:
                self._dispatch(rid, req)
            except RuntimeError as e:
                if w is not None:
                    self._finish(w, ("err", repr(e)))

    @staticmethod
    def _finish(w, result):
        w[1] = result
        w[0].set()
        if w[2] is not None:
            w[2].put(("end", None))

    def _pick(self) -> _Replica:
        live = [r for r in self.replicas if r.alive]
        if not live:
            raise RuntimeError("no live replicas")
        return min(live, key=lambda r: (len(r.inflight), r.served + len(r.inflight), r.idx))

    def _dispatch(self, rid: int, req: tuple):
        while True:
            with self._lock:
                r = self._pick()
                r.inflight[rid] = req
            try:
                with r.send_lock:
                    r.conn.send(("gen", rid) + req)
                return r
            except (OSError, EOFError, BrokenPipeError):
                self._mark_dead(r, "send failed")

    # ------------------------------------------------------------------------------ Backend API
    def generate(self, model, prompt, system="", options=None, raw=False) -> GenerateResponse:
        if self._closing:
            raise RuntimeError("router is draining")
        rid = next(self._ids)
        ev = threading.Event()
        w = [ev, None, None]  # done event, (kind, payload), stream queue
        with self._lock:
            self._waiters[rid] = w
        try:
            self._dispatch(rid, (model, prompt, system, options, raw, False))
            if not ev.wait(self.timeout_s):
                raise TimeoutError(f"request {rid} timed out")
            kind, payload = w[1]
            if kind != "ok":
                raise RuntimeError(payload)
            return GenerateResponse(**payload)
        finally:
            with self._lock:
                self._waiters.pop(rid, None)

    def generate_stream(self, model, prompt, system="", options=None, raw=False) -> Iterator[GenerateResponse]:
        if self._closing:
            raise RuntimeError("router is draining")
        rid = next(self._ids)
        w = [threading.Event(), None, queue.Queue()]
        with self._lock:
            self._waiters[rid] = w
        try:
            self._dispatch(rid, (model, prompt, system, options, raw, True))
            sent = got = 0  # chars delivered to the caller / chars of the current replica's stream
            while True:
                try:
                    kind, piece = w[2].get(timeout=self.timeout_s)
                except queue.Empty:
                    raise TimeoutError(f"request {rid} timed out") from None
                if kind == "end":
                    break
                if kind == "restart":  # re-dispatched: the new replica's stream starts over
                    got = 0
                    continue
                new = piece[max(0, sent - got):]
                got += len(piece)
                sent += len(new)
                yield GenerateResponse(model=model, response=new, done=False, done_reason="")
            kind, payload = w[1]
            if kind != "ok":
                raise RuntimeError(payload)
            final = GenerateResponse(**payload)
            full = final.response if final.response else None
            if full is not None and len(full) > sent:  # a backend that answered in one final chunk
                yield GenerateResponse(model=model, response=full[sent:], done=False, done_reason="")
            yield GenerateResponse(**{**payload, "response": ""})
        finally:
            with self._lock:
                self._waiters.pop(rid, None)

    def health(self, deep: bool = False, timeout_s: float = 1.0) -> dict:
        """Replica liveness and load; ``deep`` also asks every live replica for its engines' health (running /
        waiting / KV usage / restarts per model), waiting at most ``timeout_s`` in all."""
        out = {"ok": any(r.alive for r in self.replicas),
               "replicas": [{"id": r.idx, "alive": r.alive, "ready": r.ready, "inflight": len(r.inflight),
                             "served": r.served} for r in self.replicas]}
        if not deep:
            return out
        probes = {}
        for r, rec in zip(self.replicas, out["replicas"]):
            if not (r.alive and r.ready):
                continue
            pid = -next(self._ids)  # negative ids never collide with requests
            w = [threading.Event(), None]
            with self._lock:
                self._probes[pid] = w
            try:
                with r.send_lock:
                    r.conn.send(("health", pid))
                probes[pid] = (w, rec)
            except (OSError, EOFError, BrokenPipeError):
                with self._lock:
                    self._probes.pop(pid, None)
        t_end = time.time() + timeout_s
        for pid, (w, rec) in probes.items():
            if w[0].wait(max(0.0, t_end - time.time())):
                rec["health"] = w[1]
            with self._lock:
                self._probes.pop(pid, None)
        return out

    def models(self):
        return []

    def close(self, drain_s: float = 30.0) -> None:
        self._closing = True
        t0 = time.time()
        while any(r.inflight for r in self.replicas if r.alive) and time.time() - t0 < drain_s:
            time.sleep(0.05)
        for r in self.replicas:
            try:
                r.conn.send(("stop",))
            except (OSError, EOFError):
                pass
        for r in self.replicas:
            for p in [r.proc, *r.followers]:
                p.join(timeout=5)
                if p.is_alive():
                    p.terminate()

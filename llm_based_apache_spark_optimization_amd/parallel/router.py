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


def _worker(conn, replica: int, devices: str, kind: str, settings_kw: dict, heartbeat_s: float):
    """Replica process: build backends lazily, answer requests until told to stop."""
    if devices:
        os.environ["HIP_VISIBLE_DEVICES"] = devices  # before any HIP call in this process
    from ..config import Settings
    from ..client import FakeBackend

    if kind == "fake":
        backend = FakeBackend()
    else:
        from ..serving.service import backend_from_settings

        s = Settings(**settings_kw)
        s.dp = 1
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
            return
        if msg[0] == "stop":
            return
        if msg[0] == "gen":
            t = threading.Thread(target=serve, args=msg[1:], daemon=True)  # concurrency -> batching
            t.start()
            pool.append(t)


class _Replica:
    def __init__(self, idx: int, proc, conn):
        self.idx, self.proc, self.conn = idx, proc, conn
        self.inflight: dict = {}
        self.alive = True
        self.last_hb = time.time()
        self.ready = False  # first heartbeat seen: start-up (imports, weight load) is not a missed beat
        self.served = 0
        self.send_lock = threading.Lock()


class ReplicaRouter(Backend):
    def __init__(self, dp: int, kind: str = "hip", devices: Optional[list] = None, settings_kw: Optional[dict] = None,
                 heartbeat_s: float = 2.0, dead_after_s: float = 30.0, timeout_s: float = 300.0):
        self.kind = kind
        self.timeout_s = timeout_s
        self.dead_after_s = dead_after_s
        self._ids = itertools.count(1)
        self._lock = threading.Lock()
        self._waiters: dict = {}
        self._closing = False
        ctx = mp.get_context("spawn")
        self.replicas = []
        for i in range(dp):
            a, b = ctx.Pipe()
            dev = devices[i] if devices else (str(i) if kind != "fake" else "")
            p = ctx.Process(target=_worker, args=(b, i, dev, kind, settings_kw or {}, heartbeat_s), daemon=True)
            p.start()
            self.replicas.append(_Replica(i, p, a))
        for r in self.replicas:
            threading.Thread(target=self._reader, args=(r,), daemon=True).start()
        threading.Thread(target=self._monitor, daemon=True).start()

    @staticmethod
    def from_settings(settings) -> "ReplicaRouter":
        import dataclasses

        kw = {f.name: getattr(settings, f.name) for f in dataclasses.fields(settings)}
        tp = max(1, settings.tp)
        devices = [",".join(str(i * tp + j) for j in range(tp)) for i in range(settings.dp)]
        return ReplicaRouter(settings.dp, "fake" if settings.engine == "fake" else "hip", devices, kw,
                             timeout_s=settings.request_timeout_s)

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
                if r.alive and (not r.proc.is_alive() or hb_lost):
                    self._mark_dead(r, "process exited" if not r.proc.is_alive() else "heartbeat lost")

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

    def health(self) -> dict:
        return {"ok": any(r.alive for r in self.replicas),
                "replicas": [{"id": r.idx, "alive": r.alive, "inflight": len(r.inflight), "served": r.served}
                             for r in self.replicas]}

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
            r.proc.join(timeout=5)
            if r.proc.is_alive():
                r.proc.terminate()

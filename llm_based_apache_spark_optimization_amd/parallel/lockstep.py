"""Leader/follower lockstep for a SERVED tensor-parallel replica (SURVEY.md §2.6 P-TP behind P-DP).

The reference has exactly one model handle per process (FastAPI/app.py:19) and calls it from its
request handlers (FastAPI/app.py:85-90,105-109).  A TP replica is ``tp`` processes (one per GPU of the
replica), each holding one shard of the weights, whose kernels must issue the same collectives in the
same order.  Only the leader (TP rank 0) receives requests and runs the scheduler
(``engine.LLMEngine``); every call it makes on its ``ModelRunner`` that changes device state or
launches kernels (slot setup, prefill, decode runs, releases, graph capture) is first sent to the
followers over a pipe and then executed locally, so every rank applies the identical sequence of
runner calls — identical admissions, identical batch buckets and split plans, identical collectives.
Reads (finished flags, generated tokens) happen on the leader only: every rank holds the same
gathered logits and commits the same tokens, so there is nothing to gather back.

Engines are built through the same channel (``("build", model)``), so lazy per-model construction
(weights, TP communicators, captured graphs — all collective) also happens in lockstep.  One lock
orders the leader's calls across its engine threads; each model keeps its own TP group (own RCCL
communicator and IPC all-reduce region) and its own HIP stream on every rank.
"""
from __future__ import annotations

import contextlib
import gc
import logging
import os
import threading
from typing import Callable, Optional

import torch

log = logging.getLogger(__name__)

# ModelRunner methods that launch kernels or mutate device-resident state
MUTATORS = frozenset({"set_slot", "set_slots", "extend_tables", "release_slot", "prefill", "prefill_chunk", "decode", "set_eos", "capture",
                      "capture_all"})


class LeaderChannel:
    """Leader end: one pipe per follower; ``lock`` orders (send + local execution) across threads."""

    def __init__(self, conns: list):
        self.conns = list(conns)
        self.lock = threading.RLock()

    def send(self, msg) -> None:
        for c in self.conns:
            c.send(msg)

    def close(self) -> None:
        with self.lock:
            for c in self.conns:
                try:
                    c.send(("stop",))
                except (OSError, EOFError, BrokenPipeError):
                    pass


class LockstepRunner:
    """Leader-side proxy of a ModelRunner: mutators are mirrored to the followers, reads are local."""

    def __init__(self, runner, chan: LeaderChannel, key: str):
        object.__setattr__(self, "_runner", runner)
        object.__setattr__(self, "_chan", chan)
        object.__setattr__(self, "_key", key)

    def __getattr__(self, name):
        attr = getattr(self._runner, name)
        if name not in MUTATORS:
            return attr

        def mirrored(*args, **kwargs):
            with self._chan.lock:
                self._chan.send(("call", self._key, name, args, kwargs))
                return attr(*args, **kwargs)

        return mirrored

    def __setattr__(self, name, value):
        setattr(self._runner, name, value)


def lockstep_factory(build: Callable[[str], object], chan: Optional[LeaderChannel]) -> Callable[[str], object]:
    """Wrap an engine factory (model -> LLMEngine) for the leader of a TP replica."""
    if chan is None:
        return build

    def make(model: str):
        with chan.lock:
            chan.send(("build", model))
            eng = build(model)
        eng.runner = LockstepRunner(eng.runner, chan, model)
        return eng

    return make


def follow(conn, build: Callable[[str], object], exit_on_error: bool = True) -> None:
    """Follower loop: build engines and replay the leader's runner calls until told to stop.

    A replayed call that raises leaves this rank out of step with the leader (which ran or will run the
    same call's collectives): the follower exits non-zero (``exit_on_error``), the router sees the TP group
    lose a rank and terminates the whole replica instead of pairing later collectives wrongly."""
    engines: dict = {}
    streams: dict = {}
    while True:
        try:
            msg = conn.recv()
        except (EOFError, OSError):
            return
        kind = msg[0]
        if kind == "stop":
            return
        if kind == "build":
            model = msg[1]
            if model in engines:  # rebuild: free the old engine's weights / KV arena before the new one sizes its arena
                engines.pop(model)
                streams.pop(model, None)
                gc.collect()
                if torch.cuda.is_available():
                    torch.cuda.empty_cache()
            try:
                eng = build(model)
            except BaseException as e:  # noqa: BLE001
                _die(e, f"build {model}", exit_on_error)
                raise
            engines[model] = eng
            dev = getattr(eng.runner, "device", None)
            if dev is not None and torch.device(dev).type == "cuda":
                s = torch.cuda.Stream(device=dev)  # mirrors the leader's per-engine stream
                s.wait_stream(torch.cuda.current_stream(dev))
                streams[model] = s
            continue
        if kind == "call":
            _, model, name, args, kwargs = msg
            s = streams.get(model)
            ctx = torch.cuda.stream(s) if s is not None else contextlib.nullcontext()
            try:
                with ctx:
                    getattr(engines[model].runner, name)(*args, **kwargs)
            except BaseException as e:  # noqa: BLE001
                _die(e, name, exit_on_error)
                raise
            continue
        log.warning("follower: unknown message %r", kind)


def _die(e: BaseException, what: str, exit_on_error: bool) -> None:
    log.error("TP follower: %s failed (%r); leaving the replica", what, e)
    if exit_on_error:
        os._exit(71)

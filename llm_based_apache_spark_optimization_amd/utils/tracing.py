"""Per-request spans (queue, tokenize, prefill, decode, SQL, history) with optional JSONL export.

Enabled with ``LSA_TRACE=1`` (or ``Settings.trace``); spans are always fed to the metrics registry as
``lsa_stage_seconds{stage=...}`` so /metrics shows the per-stage latency split either way.  GPU kernel
traces come from ``rocprofv3 --kernel-trace --stats`` (scripts/profile_bench.sh).
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
import uuid

from .metrics import REGISTRY

_lock = threading.Lock()
_path = os.environ.get("LSA_TRACE_FILE", "lsa_trace.jsonl")
ENABLED = os.environ.get("LSA_TRACE", "0").lower() in ("1", "true", "yes")


def new_request_id() -> str:
    return uuid.uuid4().hex[:16]


@contextlib.contextmanager
def span(stage: str, request_id: str = "", **attrs):
    t0 = time.perf_counter()
    err = None
    try:
        yield
    except BaseException as e:  # noqa: BLE001
        err = repr(e)
        raise
    finally:
        dt = time.perf_counter() - t0
        REGISTRY.observe("lsa_stage_seconds", dt, "per-stage latency", stage=stage)
        if ENABLED:
            rec = {"ts": time.time(), "request_id": request_id, "stage": stage, "seconds": dt, **attrs}
            if err:
                rec["error"] = err
            with _lock, open(_path, "a") as f:
                f.write(json.dumps(rec) + "\n")


def record(stage: str, seconds: float, request_id: str = "", **attrs) -> None:
    """A span measured elsewhere (e.g. the engine's per-request queue / prefill / decode / detok phases,
    known only when the request completes): same metric and JSONL record as ``span``."""
    labels = {k: v for k, v in attrs.items() if k == "model"}
    REGISTRY.observe("lsa_stage_seconds", max(0.0, seconds), "per-stage latency", stage=stage, **labels)
    if ENABLED:
        rec = {"ts": time.time(), "request_id": request_id, "stage": stage, "seconds": seconds, **attrs}
        with _lock, open(_path, "a") as f:
            f.write(json.dumps(rec) + "\n")

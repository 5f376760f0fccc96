"""Service wiring: model backend + SQL executor + history store + pipeline from one Settings."""
from __future__ import annotations

import dataclasses
import logging

from ..client import Backend, EngineService, FakeBackend, RemoteBackend
from ..config import Settings
from .executor import make_executor
from .history import HistoryStore
from .pipeline import Pipeline, StatusBoard

log = logging.getLogger(__name__)


def engine_factory(settings: Settings, tp_factory=None):
    """model name -> LLMEngine on this process's GPU (fp8 for the NL->SQL model when configured).
    ``tp_factory()`` -> this rank's TPGroup for the model being built (TP replicas, parallel/router.py)."""

    def build(model: str):
        from ..engine import build_engine

        dtype = settings.dtype if model == settings.nl2sql_model else settings.explain_dtype
        tp = tp_factory() if tp_factory is not None else None
        log.info("building engine %s (%s, max_batch=%d, tp=%d)", model, dtype, settings.max_batch,
                 tp.size if tp is not None else 1)
        # two models co-serve one GPU: each engine's KV arena takes a share of the memory free at its build
        return build_engine(model, checkpoint=settings.checkpoint_dir if model == settings.nl2sql_model else None,
                            dtype=dtype, max_slots=settings.max_batch, max_model_len=settings.max_model_len,
                            kv_memory_fraction=settings.kv_memory_fraction, warm_graphs=True, tp=tp,
                            prefill_chunk=settings.prefill_chunk, kv_dtype=settings.kv_dtype,
                            max_new_cap=settings.max_new_cap or None,
                            kv_reserve_tokens=settings.kv_reserve_tokens)

    return build


def backend_from_settings(settings: Settings) -> Backend:
    defaults = {"temperature": settings.temperature, "top_k": settings.top_k, "top_p": settings.top_p,
                "num_predict": settings.max_new_tokens}
    if settings.engine == "fake":
        return FakeBackend()
    if settings.engine == "remote":
        return RemoteBackend(settings.remote_url, settings.request_timeout_s)
    if settings.dp > 1 or settings.tp > 1:  # replica processes (TP groups need one process per GPU)
        from ..parallel.router import ReplicaRouter

        return ReplicaRouter.from_settings(settings)
    return EngineService(engine_factory(settings), defaults=defaults, timeout_s=settings.request_timeout_s)


@dataclasses.dataclass
class AppContext:
    settings: Settings
    backend: Backend
    pipeline: Pipeline
    history: HistoryStore
    status: StatusBoard


def make_context(settings: Settings | None = None, backend: Backend | None = None, executor=None,
                 history: HistoryStore | None = None) -> AppContext:
    settings = settings or Settings()
    settings.ensure_dirs()
    backend = backend or backend_from_settings(settings)
    history = history or HistoryStore(settings.history_dsn)
    status = StatusBoard()
    pipe = Pipeline(backend, executor or make_executor(settings.sql_backend), history, settings, status)
    return AppContext(settings, backend, pipe, history, status)

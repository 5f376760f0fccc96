"""FastAPI JSON service.

Reference-compatible route (FastAPI/app.py:62-144): ``POST /process-data/`` with body
``{"input_text": str, "file_name": str}``; the CSV is resolved under the configured input directory;
responses keep the reference's keys and its HTTP-200-with-"error" convention:

* success  ``{"message": "Query executed successfully!", "input_file_name", "input_data", "sql_query",
  "output_file"}``
* SQL error ``{"error": "SQL execution failed", "sql_query", "error_details"}`` (LLM#2's explanation)
* missing  ``{"error": "CSV file not found at <path>"}``

North-star endpoints (BASELINE.json): ``POST /nl2sql`` and ``POST /explain_error``.  Plus an
Ollama-compatible ``POST /api/generate`` / ``GET /api/tags`` (so ``ollama``-style clients, including
the reference's own harness pointed at this host, work unchanged), ``/health``, ``/ready``,
``/metrics`` (Prometheus) and ``/status/{request_id}``.

Handlers are plain ``def`` (run in FastAPI's threadpool): the reference's ``async def`` handlers
made blocking calls and serialised every request on the event loop (SURVEY.md §2.6 P-DP); here
concurrent requests reach the engine together and share decode steps.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from pydantic import BaseModel

from .. import prompts
from ..client import EngineUnavailable
from ..utils.metrics import REGISTRY, record_generation
from ..utils.tracing import new_request_id
from .pipeline import resolve_input
from .service import AppContext, make_context


class InputString(BaseModel):
    input_text: str
    file_name: str


class NL2SQLRequest(BaseModel):
    question: Optional[str] = None
    input_text: Optional[str] = None
    table_schema: Optional[str] = None
    schema_text: Optional[str] = None
    file_name: Optional[str] = None
    options: Optional[dict] = None


class ExplainRequest(BaseModel):
    error_message: str
    options: Optional[dict] = None


class GenerateRequest(BaseModel):
    model: str
    prompt: str = ""
    system: str = ""
    options: Optional[dict] = None
    stream: bool = False
    raw: bool = False


def create_app(ctx: Optional[AppContext] = None) -> FastAPI:
    ctx = ctx or make_context()
    app = FastAPI(title="MI355X NL->SQL / Spark-error service")
    app.state.ctx = ctx
    s = ctx.settings

    @app.exception_handler(EngineUnavailable)
    def engine_down(request: Request, exc: EngineUnavailable):
        # a dead engine answers at once (SURVEY.md §5 failure detection) instead of after the request timeout
        REGISTRY.inc("lsa_requests_total", 1, "requests", route=request.url.path.strip("/"), outcome="unavailable")
        return JSONResponse(status_code=503, content={"error": "engine unavailable", "detail": str(exc)})

    @app.post("/process-data/")
    def modify_string(data: InputString):
        t0 = time.perf_counter()
        file_path = resolve_input(s.input_dir, data.file_name)
        if file_path is None:
            REGISTRY.inc("lsa_requests_total", 1, "requests", route="process-data", outcome="bad_name")
            return {"error": "Invalid file name: " + data.file_name}
        if not os.path.exists(file_path):
            REGISTRY.inc("lsa_requests_total", 1, "requests", route="process-data", outcome="not_found")
            return {"error": "CSV file not found at " + file_path}
        res = ctx.pipeline.run(file_path, data.file_name, data.input_text,
                               output_name=lambda ts: f"{ts}_{os.path.basename(file_path)}.csv")
        REGISTRY.observe("lsa_request_seconds", time.perf_counter() - t0, "e2e latency", route="process-data")
        if not res.ok:
            REGISTRY.inc("lsa_requests_total", 1, "requests", route="process-data", outcome="sql_error")
            return {"error": "SQL execution failed", "sql_query": res.sql_query, "error_details": res.explanation}
        REGISTRY.inc("lsa_requests_total", 1, "requests", route="process-data", outcome="ok")
        return {
            "message": "Query executed successfully!",
            "input_file_name": data.file_name,
            "input_data": data.input_text,
            "sql_query": res.sql_query,
            "output_file": res.output_file,
        }

    @app.post("/nl2sql")
    def nl2sql(req: NL2SQLRequest):
        t0 = time.perf_counter()
        question = req.question or req.input_text
        if not question:
            raise HTTPException(422, "question (or input_text) is required")
        schema = req.table_schema or req.schema_text
        if schema is None and req.file_name:
            path = resolve_input(s.input_dir, req.file_name)
            if path is None:
                raise HTTPException(400, "invalid file_name: " + req.file_name)
            if not os.path.exists(path):
                return {"error": "CSV file not found at " + path}
            table = ctx.pipeline.executor.table_of(ctx.pipeline.executor.load_csv(path))
            schema = prompts.table_schema_text(table.dtypes)
        if schema is None:
            raise HTTPException(422, "table_schema or file_name is required")
        rid = new_request_id()
        r = ctx.pipeline.nl2sql(schema, question, req.options, rid)
        dt = time.perf_counter() - t0
        REGISTRY.observe("lsa_request_seconds", dt, "e2e latency", route="nl2sql")
        REGISTRY.inc("lsa_requests_total", 1, "requests", route="nl2sql", outcome="ok")
        return {"sql_query": r.response, "model": r.model, "request_id": rid, "table_schema": schema,
                "eval_count": r.eval_count, "eval_duration": r.eval_duration,
                "prompt_eval_count": r.prompt_eval_count, "total_duration": r.total_duration, "latency_s": dt}

    @app.post("/explain_error")
    def explain_error(req: ExplainRequest):
        t0 = time.perf_counter()
        rid = new_request_id()
        r = ctx.pipeline.explain(req.error_message, req.options, rid)
        dt = time.perf_counter() - t0
        REGISTRY.observe("lsa_request_seconds", dt, "e2e latency", route="explain_error")
        REGISTRY.inc("lsa_requests_total", 1, "requests", route="explain_error", outcome="ok")
        return {"explanation": r.response, "model": r.model, "request_id": rid, "eval_count": r.eval_count,
                "eval_duration": r.eval_duration, "prompt_eval_count": r.prompt_eval_count,
                "total_duration": r.total_duration, "latency_s": dt}

    @app.post("/api/generate")
    def api_generate(req: GenerateRequest):
        if req.stream:  # Ollama's NDJSON framing: response pieces as decoded, then the done chunk
            chunks = ctx.backend.generate_stream(req.model, req.prompt, req.system, req.options, req.raw)

            def ndjson():
                for c in chunks:
                    if c.done:
                        record_generation(c, "api_generate")
                    yield json.dumps(c.to_dict()) + "\n"
            return StreamingResponse(ndjson(), media_type="application/x-ndjson")
        r = ctx.backend.generate(req.model, req.prompt, req.system, req.options, req.raw)
        record_generation(r, "api_generate")
        return r.to_dict()

    @app.get("/api/tags")
    def api_tags():
        return {"models": [{"name": m, "model": m} for m in (ctx.backend.models() or
                                                              [s.nl2sql_model, s.explain_model])]}

    @app.get("/api/version")
    def api_version():
        return {"version": "lsa-mi355x-0.1"}

    @app.get("/status/{request_id}")
    def status(request_id: str):
        return ctx.status.get(request_id)

    @app.get("/health")
    def health():
        return ctx.backend.health()

    @app.get("/ready")
    def ready():
        h = ctx.backend.health()
        if not h.get("ok", False):
            raise HTTPException(503, "engine not healthy")
        return {"ready": True}

    @app.get("/metrics", response_class=PlainTextResponse)
    def metrics():
        export_backend_gauges(ctx.backend)
        return REGISTRY.render()

    return app


def export_backend_gauges(backend) -> None:
    """Engine gauges (running / waiting / KV usage / restarts per model) and, under DP, per-replica load
    (alive, in-flight, served) plus each replica's engine gauges (``ReplicaRouter.health(deep=True)``)."""
    try:
        h = backend.health(deep=True)
    except Exception:  # noqa: BLE001 - metrics must render even when the backend is down
        h = {}

    def engines(eng: dict, **lbl):
        for m, e in (eng or {}).items():
            REGISTRY.set("lsa_engine_running", e.get("running", 0), "running requests", model=m, **lbl)
            REGISTRY.set("lsa_engine_waiting", e.get("waiting", 0), "queued requests", model=m, **lbl)
            REGISTRY.set("lsa_engine_kv_usage", e.get("kv_usage", 0.0), "KV cache fraction in use", model=m, **lbl)
            REGISTRY.set("lsa_engine_alive", 1.0 if e.get("alive", True) else 0.0, "engine loop alive", model=m, **lbl)
            REGISTRY.set("lsa_engine_restarts", e.get("restarts", 0) + e.get("rebuilds", 0),
                         "engine recoveries (loop restarts + rebuilds)", model=m, **lbl)
    engines(h.get("engines"))
    for r in h.get("replicas") or []:
        rid = str(r.get("id"))
        REGISTRY.set("lsa_replica_alive", 1.0 if r.get("alive") else 0.0, "DP replica alive", replica=rid)
        REGISTRY.set("lsa_replica_inflight", r.get("inflight", 0), "requests in flight on the replica", replica=rid)
        REGISTRY.set("lsa_replica_served", r.get("served", 0), "requests served by the replica", replica=rid)
        engines((r.get("health") or {}).get("engines"), replica=rid)


def main(argv=None) -> None:  # pragma: no cover - server entry point
    import argparse

    import uvicorn

    from ..config import Settings
    from ..utils import setup_logging

    ap = argparse.ArgumentParser(description="FastAPI NL->SQL service on MI355X")
    Settings.add_cli(ap)
    settings = Settings.from_cli(ap.parse_args(argv))
    setup_logging(settings.log_level)
    uvicorn.run(create_app(make_context(settings)), host=settings.host, port=settings.fastapi_port)


if __name__ == "__main__":  # pragma: no cover
    main()

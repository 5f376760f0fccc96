"""Request orchestration shared by the FastAPI and Flask apps (the reference's L2 layer).

schema -> NL->SQL (LLM#1) -> execute -> explain-on-error (LLM#2) -> persist, exactly the flow of
``modify_string`` (FastAPI/app.py:62-144) and ``process_data`` (Flask/app.py:75-172), with the
reference's latent races fixed: per-request ids, a per-request status board (the
reference kept one process-global dict, Flask/app.py:59-72), per-request output timestamps (the
reference stamped once at import, FastAPI/app.py:12-13, so successive requests overwrote each
other's files) and no shared temp directory.
"""
from __future__ import annotations

import dataclasses
import datetime as _dt
import logging
import os
import threading
import time
from collections import OrderedDict
from typing import Callable, Optional

from .. import prompts
from ..utils.metrics import REGISTRY, record_generation
from ..utils.tracing import new_request_id, span
from .executor import SQLExecutionError, write_csv
from .history import HistoryStore

log = logging.getLogger(__name__)

# the reference's progress strings (Flask/app.py:79-165) — kept verbatim for UI compatibility
ST_UPLOAD = "Uploading file..."
ST_LOAD = "CSV file loading into Spark."
ST_GEN = "Generating SQL query..."
ST_GEN_OK = "SQL query generated successfully."
ST_EXEC = "Executing query in Spark..."
ST_CSV = "Saving results to CSV..."
ST_DB = "Saving results to MySQL..."
ST_ERR = "Error occurred"
ST_FIX = "Trying to resolve error..."
ST_FIXED = "Error resolved"


class StatusBoard:
    """Per-request progress (``idle`` / ``running`` / ``done``) + the latest request for the
    reference's parameterless ``GET /status``."""

    def __init__(self, keep: int = 1024):
        self._lock = threading.Lock()
        self._jobs: "OrderedDict[str, dict]" = OrderedDict()
        self._latest: Optional[str] = None
        self.keep = keep

    def update(self, job: str, message: str, status: str = "running", **extra) -> None:
        with self._lock:
            d = self._jobs.setdefault(job, {"status": "idle", "message": "Waiting for input"})
            d.update(status=status, message=message, **extra)
            self._jobs.move_to_end(job)
            self._latest = job
            while len(self._jobs) > self.keep:
                self._jobs.popitem(last=False)

    def get(self, job: Optional[str] = None) -> dict:
        with self._lock:
            key = job or self._latest
            if key is None or key not in self._jobs:
                return {"status": "idle", "message": "Waiting for input"}
            return dict(self._jobs[key], job=key)


@dataclasses.dataclass
class JobResult:
    ok: bool
    request_id: str
    input_file_name: str
    input_text: str
    table_schema: str = ""
    sql_query: str = ""
    output_file: str = ""
    error_message: str = ""
    explanation: str = ""
    timings: dict = dataclasses.field(default_factory=dict)


def timestamp() -> str:
    return _dt.datetime.now().strftime("%Y_%m_%d_%H_%M_%S")


def unique_path(path: str) -> str:
    """Atomically reserve ``path`` (or ``base_N.ext``) with O_CREAT|O_EXCL: concurrent requests that
    compute the same name in the same second never share a file."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    base, ext = os.path.splitext(path)
    cand, i = path, 0
    while True:
        try:
            os.close(os.open(cand, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644))
            return cand
        except FileExistsError:
            i += 1
            cand = f"{base}_{i}{ext}"


def resolve_input(input_dir: str, name: str) -> Optional[str]:
    """``name`` resolved under ``input_dir``, or None when it would leave that directory (absolute
    paths, ``..`` components, symlinks pointing outside).  The reference joined the untrusted
    ``file_name`` onto its input directory unchecked (FastAPI/app.py:68)."""
    if not name or "\x00" in name or os.path.isabs(name):
        return None
    root = os.path.realpath(input_dir)
    path = os.path.realpath(os.path.join(root, name))
    if os.path.commonpath([root, path]) != root or path == root:
        return None
    return path


class Pipeline:
    def __init__(self, backend, executor, history: HistoryStore, settings, status: Optional[StatusBoard] = None):
        self.backend = backend
        self.executor = executor
        self.history = history
        self.settings = settings
        self.status = status or StatusBoard()

    # ------------------------------------------------------------------------------- LLM calls
    def nl2sql(self, table_schema: str, question: str, options: Optional[dict] = None, rid: str = ""):
        with span("nl2sql", rid):
            res = self.backend.generate(self.settings.nl2sql_model, question,
                                        system=prompts.nl2sql_system(table_schema), options=options)
        record_generation(res, "nl2sql")
        return res

    def explain(self, error_message: str, options: Optional[dict] = None, rid: str = ""):
        with span("explain_error", rid):
            res = self.backend.generate(self.settings.explain_model, prompts.explain_prompt(error_message),
                                        system=prompts.EXPLAIN_SYSTEM, options=options)
        record_generation(res, "explain_error")
        return res

    # ------------------------------------------------------------------------------- full job
    def run(self, file_path: str, file_name: str, input_text: str, output_name: Callable[[str], str],
            job: Optional[str] = None, history_name: Optional[Callable[[str], str]] = None,
            options: Optional[dict] = None) -> JobResult:
        rid = job or new_request_id()
        st = lambda m: self.status.update(rid, m)  # noqa: E731
        out = JobResult(False, rid, file_name, input_text)
        t0 = time.perf_counter()
        session = None
        try:
            st(ST_LOAD)
            with span("load_csv", rid):
                loaded = self.executor.load_csv(file_path)
                table = self.executor.table_of(loaded)
            out.table_schema = prompts.table_schema_text(table.dtypes)
            st(ST_GEN)
            out.sql_query = self.nl2sql(out.table_schema, input_text, options, rid).response
            st(ST_GEN_OK)
            st(ST_EXEC)
            with span("sql", rid):
                session = self.executor.session(loaded)
                result = session.sql(out.sql_query)
            st(ST_CSV)
            ts = timestamp()
            out.output_file = unique_path(os.path.join(self.settings.output_dir, output_name(ts)))
            with span("write_csv", rid):
                write_csv(result, out.output_file)
            st(ST_DB)
            with span("history", rid):
                self.history.insert(file_name, input_text, out.sql_query,
                                    history_name(out.output_file) if history_name else out.output_file)
            out.ok = True
            REGISTRY.inc("lsa_jobs_total", 1, "pipeline jobs", outcome="ok")
        except SQLExecutionError as e:
            out.error_message = str(e)
            self._explain_into(out, options, rid)
        except Exception as e:  # noqa: BLE001 - the Flask reference routes every error to the explainer
            out.error_message = str(e) or repr(e)
            log.exception("job %s failed", rid)
            self._explain_into(out, options, rid)
        finally:
            if session is not None:
                session.close()
            out.timings["total_s"] = time.perf_counter() - t0
            REGISTRY.observe("lsa_job_seconds", out.timings["total_s"], "pipeline job latency",
                             outcome="ok" if out.ok else "error")
            self.status.update(rid, ST_FIXED if not out.ok else ST_DB, status="done")
        return out

    def _explain_into(self, out: JobResult, options, rid: str) -> None:
        REGISTRY.inc("lsa_jobs_total", 1, "pipeline jobs", outcome="sql_error")
        self.status.update(rid, ST_ERR)
        self.status.update(rid, ST_FIX)
        try:
            out.explanation = self.explain(out.error_message, options, rid).response
        except Exception as e:  # noqa: BLE001 - the explainer itself failed (engine down, timeout)
            log.error("explain failed: %s", e)
            out.explanation = f"(explanation unavailable: {e})"
        self.status.update(rid, ST_FIXED)

"""One settings object for the whole service (env vars ``LSA_*`` + CLI flags).

The reference hard-codes everything (SURVEY.md §5 "Config / flag system"): WSL input/output paths
(FastAPI/app.py:68,118; Flask/app.py:19-20), the MySQL DSN 172.23.131.215 root/root db ``project``
(FastAPI/app.py:31-36), model names (FastAPI/app.py:86,106), the Flask secret (Flask/app.py:12),
host/port (FastAPI/app.py:148, Flask default 5000) and the history page size 8 (Flask/app.py:214).
Defaults here keep the reference behaviour (model names, page size, ports) while making every value
configurable.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from typing import Optional


def _env(name: str, default, cast=str):
    v = os.environ.get("LSA_" + name)
    if v is None:
        return default
    if cast is bool:
        return v.lower() in ("1", "true", "yes", "on")
    return cast(v)


@dataclasses.dataclass
class Settings:
    # paths
    input_dir: str = dataclasses.field(default_factory=lambda: _env("INPUT_DIR", os.path.abspath("data/Input")))
    output_dir: str = dataclasses.field(default_factory=lambda: _env("OUTPUT_DIR", os.path.abspath("data/Output")))
    # persistence: "sqlite:///path.db" (default) or "mysql://user:pw@host/db"
    history_dsn: str = dataclasses.field(default_factory=lambda: _env("HISTORY_DSN", "sqlite:///data/history.db"))
    history_page_size: int = dataclasses.field(default_factory=lambda: _env("HISTORY_PAGE_SIZE", 8, int))
    # SQL execution backend: "sqlite" (default) | "spark" (needs pyspark)
    sql_backend: str = dataclasses.field(default_factory=lambda: _env("SQL_BACKEND", "sqlite"))
    # models
    nl2sql_model: str = dataclasses.field(default_factory=lambda: _env("NL2SQL_MODEL", "duckdb-nsql"))
    explain_model: str = dataclasses.field(default_factory=lambda: _env("EXPLAIN_MODEL", "llama3.2"))
    # engine: "hip" (MI355X engine), "fake" (deterministic test engine), "remote" (HTTP to another server)
    engine: str = dataclasses.field(default_factory=lambda: _env("ENGINE", "hip"))
    remote_url: str = dataclasses.field(default_factory=lambda: _env("REMOTE_URL", "http://127.0.0.1:8000"))
    checkpoint_dir: Optional[str] = dataclasses.field(default_factory=lambda: _env("CHECKPOINT_DIR", None))
    dtype: str = dataclasses.field(default_factory=lambda: _env("DTYPE", "bf16"))
    explain_dtype: str = dataclasses.field(default_factory=lambda: _env("EXPLAIN_DTYPE", "bf16"))
    # paged KV cache dtype of every engine: "bf16" | "fp8" (e4m3 rows + per-row scales, ops.KV_FP8)
    kv_dtype: str = dataclasses.field(default_factory=lambda: _env("KV_DTYPE", "bf16"))
    tp: int = dataclasses.field(default_factory=lambda: _env("TP", 1, int))
    dp: int = dataclasses.field(default_factory=lambda: _env("DP", 1, int))
    max_batch: int = dataclasses.field(default_factory=lambda: _env("MAX_BATCH", 32, int))
    max_model_len: int = dataclasses.field(default_factory=lambda: _env("MAX_MODEL_LEN", 4096, int))
    # share of the free GPU memory each engine's paged KV arena takes when it is built (two co-served
    # models: the first gets 45 %, the second 45 % of what is left)
    kv_memory_fraction: float = dataclasses.field(default_factory=lambda: _env("KV_MEMORY_FRACTION", 0.45, float))
    # default num_predict of a request that sets none: -1 = Ollama's default, generate until EOS or the context
    # window (the reference's option-less ollama.generate calls, FastAPI/app.py:85-90,105-109)
    max_new_tokens: int = dataclasses.field(default_factory=lambda: _env("MAX_NEW_TOKENS", -1, int))
    # server safety cap on generated tokens per request (0 = the model context window); far above any
    # typical NL->SQL or explanation answer, it only bounds a model that never emits EOS
    max_new_cap: int = dataclasses.field(default_factory=lambda: _env("MAX_NEW_CAP", 0, int))
    # KV reservation at admission: prompt + this many generated tokens; decode runs grow the tables block by block
    # and an exhausted arena preempts the youngest request (-1 = reserve prompt + max_new up front)
    kv_reserve_tokens: int = dataclasses.field(default_factory=lambda: _env("KV_RESERVE_TOKENS", 64, int))
    # chunked-prefill interleave: prompt tokens prefilled per engine iteration (0 = whole prompts); longer
    # prompts stall the running decode batch one chunk at a time.  The budget also caps prefill throughput
    # (one chunk per decode run): 512 collapsed co-serving at 16 QPS (nl2sql p50 0.56 -> 3.4 s), 2048 does not
    # (scripts/gpu_r2_serving_ab.sh)
    prefill_chunk: int = dataclasses.field(default_factory=lambda: _env("PREFILL_CHUNK", 2048, int))
    # sampling defaults: greedy (the reference sampled at Ollama defaults; pass options to match)
    temperature: float = dataclasses.field(default_factory=lambda: _env("TEMPERATURE", 0.0, float))
    top_k: int = dataclasses.field(default_factory=lambda: _env("TOP_K", 40, int))
    top_p: float = dataclasses.field(default_factory=lambda: _env("TOP_P", 0.9, float))
    request_timeout_s: float = dataclasses.field(default_factory=lambda: _env("REQUEST_TIMEOUT", 300.0, float))
    # servers
    host: str = dataclasses.field(default_factory=lambda: _env("HOST", "127.0.0.1"))
    fastapi_port: int = dataclasses.field(default_factory=lambda: _env("FASTAPI_PORT", 8000, int))
    flask_port: int = dataclasses.field(default_factory=lambda: _env("FLASK_PORT", 5000, int))
    secret_key: str = dataclasses.field(default_factory=lambda: _env("SECRET_KEY", os.urandom(16).hex()))
    log_level: str = dataclasses.field(default_factory=lambda: _env("LOG_LEVEL", "INFO"))
    trace: bool = dataclasses.field(default_factory=lambda: _env("TRACE", False, bool))

    def ensure_dirs(self) -> None:
        os.makedirs(self.input_dir, exist_ok=True)
        os.makedirs(self.output_dir, exist_ok=True)
        if self.history_dsn.startswith("sqlite:///"):
            d = os.path.dirname(self.history_dsn[len("sqlite:///"):])
            if d:
                os.makedirs(d, exist_ok=True)

    @staticmethod
    def add_cli(ap: argparse.ArgumentParser) -> None:
        for f in dataclasses.fields(Settings):
            t = {int: int, float: float, bool: None}.get(type(Settings().__getattribute__(f.name)), str)
            flag = "--" + f.name.replace("_", "-")
            if t is None:
                ap.add_argument(flag, action="store_true", default=None)
            else:
                ap.add_argument(flag, type=t, default=None)

    @staticmethod
    def from_cli(ns: argparse.Namespace) -> "Settings":
        s = Settings()
        for f in dataclasses.fields(Settings):
            v = getattr(ns, f.name, None)
            if v is not None:
                setattr(s, f.name, v)
        return s

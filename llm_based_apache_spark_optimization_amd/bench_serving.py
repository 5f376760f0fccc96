"""Co-serving load benchmark: BASELINE.json config 5.

duckdb-nsql-7B (fp8 weights by default) and Llama-3.2-3B-Instruct (bf16) are served from ONE process
and ONE MI355X behind the real FastAPI app (uvicorn on 127.0.0.1, real HTTP).  A load generator posts
``/nl2sql`` and ``/explain_error`` requests at a fixed Poisson rate (``--qps``), with a fixed fraction
of explain requests carrying a long synthetic Spark ``AnalysisException`` (logical plan included, like
the reference's error strings).  Outputs are fixed-length (``num_predict`` +
``ignore_eos``; the weights are random-init, so EOS timing would be meaningless) and greedy.

The reference has no load test at all; its only timings are ``time.time()`` around single
``ollama.generate`` calls (Model_Evaluation_&_Comparision.py:20,42-43) — 5.24 s p50 for duckdb-nsql
and 22.75 s for the explain path.

    python -m llm_based_apache_spark_optimization_amd.bench_serving --qps 8 --duration 30

prints one JSON line: achieved rate, completed / failed requests, output tokens/s, and p50 / p90 / p99
end-to-end latency per route (client-side wall clock around each HTTP request).
"""
from __future__ import annotations

import argparse
import json
import sys
import os
import random
import socket
import statistics
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Optional

COLS = ["VendorID bigint", "tpep_pickup_datetime timestamp", "tpep_dropoff_datetime timestamp",
        "passenger_count double", "trip_distance double", "RatecodeID double", "store_and_fwd_flag string",
        "PULocationID bigint", "DOLocationID bigint", "payment_type bigint", "fare_amount double",
        "extra double", "mta_tax double", "tip_amount double", "tolls_amount double",
        "improvement_surcharge double", "total_amount double", "congestion_surcharge double",
        "airport_fee double", "Incubation_Center string", "Name_of_startup string", "Sector string"]
QUESTIONS = ["get all trips with a fare above 50 dollars", "average tip by payment type",
             "count rides per vendor ordered by count", "total revenue per pickup location",
             "longest trip distance for each passenger count", "list startups in the fintech sector"]


def synthetic_schema(rng: random.Random, ncols: int = 14) -> str:
    cols = rng.sample(COLS, min(ncols, len(COLS)))
    return "\n".join(f"{c.split()[0]} ({c.split()[1]})" for c in cols)


def synthetic_spark_error(rng: random.Random, approx_tokens: int = 1024, chars_per_token: float = 4.0) -> str:
    """A Spark AnalysisException with a logical plan, padded to roughly ``approx_tokens`` tokens."""
    col = rng.choice(["fare", "tip", "vendor", "distance", "pickup_zone"])
    head = (f"[UNRESOLVED_COLUMN.WITH_SUGGESTION] A column or function parameter with name `{col}` cannot be "
            f"resolved. Did you mean one of the following? [`fare_amount`, `tip_amount`, `VendorID`, "
            f"`trip_distance`, `PULocationID`].; line 1 pos 32;\n'Project [*]\n+- 'Filter ('{col} > 50)\n")
    lines = [head]
    i = 0
    while sum(len(x) for x in lines) < approx_tokens * chars_per_token:
        lines.append(f"   +- SubqueryAlias temp_view_{i}\n      +- View (`temp_view_{i}`, [VendorID#{17 + i}L, "
                     f"tpep_pickup_datetime#{18 + i}, fare_amount#{27 + i}, tip_amount#{30 + i}, "
                     f"total_amount#{33 + i}])\n         +- Relation [VendorID#{17 + i}L,fare_amount#{27 + i}] csv\n")
        i += 1
    return "".join(lines)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pct(xs: list, q: float) -> Optional[float]:
    if not xs:
        return None
    xs = sorted(xs)
    k = min(len(xs) - 1, max(0, int(round(q * (len(xs) - 1)))))
    return round(xs[k], 4)


class Server:
    """The FastAPI app on uvicorn in a background thread (real sockets, real HTTP)."""

    def __init__(self, app, port: int):
        import uvicorn

        self.port = port
        self.server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning",
                                                    access_log=False))
        self.thread = threading.Thread(target=self.server.run, daemon=True)

    def __enter__(self):
        self.thread.start()
        t0 = time.time()
        while not self.server.started:
            if time.time() - t0 > 60 or not self.thread.is_alive():
                raise RuntimeError("uvicorn did not start")
            time.sleep(0.05)
        return self

    def __exit__(self, *exc):
        self.server.should_exit = True
        self.thread.join(timeout=10)


def run(args) -> dict:
    import anyio
    import httpx

    from .config import Settings
    from .serving.fastapi_app import create_app
    from .serving.service import make_context

    work = tempfile.mkdtemp(prefix="lsa_serving_")
    settings = Settings(engine=args.engine, dtype=args.nl2sql_dtype, explain_dtype=args.explain_dtype,
                        max_batch=args.max_batch, max_model_len=args.max_model_len, temperature=0.0,
                        input_dir=os.path.join(work, "in"), output_dir=os.path.join(work, "out"),
                        history_dsn=f"sqlite:///{work}/history.db")
    ctx = make_context(settings)
    app = create_app(ctx)

    async def _widen_threadpool():  # FastAPI runs sync endpoints on anyio worker threads (default 40)
        anyio.to_thread.current_default_thread_limiter().total_tokens = max(40, args.concurrency)

    app.router.on_startup.append(_widen_threadpool)
    port = _free_port()
    rng = random.Random(args.seed)
    # --option-less: the reference's call shape (no num_predict): every request may run to its context window, and
    # the engines reserve KV lazily (prompt + one block at admission, growth per decode run, youngest preempted)
    opts = {"temperature": 0.0} if args.option_less else {"num_predict": args.new_tokens, "ignore_eos": True,
                                                           "temperature": 0.0}
    # random-init engines tokenize bytes (no tokenizer files offline): 1 char = 1 token there, ~4 with
    # the real Llama-3 BPE, so size the error text in tokens of the tokenizer actually serving it
    from .models import get_spec, tokenizer_for

    cpt = 1.0 if type(tokenizer_for(get_spec("llama3.2"))).__name__ == "ByteTokenizer" else 4.0

    def make_request(i: int):
        if rng.random() < args.explain_frac:
            return "explain_error", {"error_message": synthetic_spark_error(rng, args.explain_tokens, cpt),
                                     "options": opts}
        return "nl2sql", {"table_schema": synthetic_schema(rng), "question": rng.choice(QUESTIONS), "options": opts}

    with Server(app, port):
        base = f"http://127.0.0.1:{port}"
        limits = httpx.Limits(max_connections=args.concurrency, max_keepalive_connections=args.concurrency)
        with httpx.Client(base_url=base, timeout=args.timeout, limits=limits) as cl:
            # warm-up: builds both engines (weights, KV arena) and captures their decode graphs
            t0 = time.perf_counter()
            for route, body in (make_request(0), ("nl2sql", {"table_schema": "a (int)", "question": "q",
                                                             "options": opts}),
                                ("explain_error", {"error_message": synthetic_spark_error(rng, 256, cpt),
                                                   "options": opts})):
                cl.post("/" + route, json=body).raise_for_status()
            warm_s = time.perf_counter() - t0

            phases = []
            for q in str(args.qps).split(","):
                phases.append(_phase(cl, args, float(q), rng, make_request))
                # progress on stderr (long multi-phase runs stay visibly alive)
                print(f"phase qps={q}: {phases[-1].get('output_tokens_per_sec')} tok/s", file=sys.stderr, flush=True)
    # per-engine admission / KV statistics (peak concurrently running requests, lazy-KV growth and preemptions)
    eng_stats = {}
    for m, lp in getattr(ctx.backend, "_loops", {}).items():
        st = getattr(getattr(lp, "engine", None), "stats", None)
        if st:
            r = lp.engine.runner
            eng_stats[m] = {k: st.get(k) for k in ("requests", "peak_running", "preempted", "kv_grown_blocks")}
            eng_stats[m].update(kv_blocks=getattr(r, "num_kv_blocks", None), max_slots=getattr(r, "max_slots", None))
    for p in phases:
        p.update(engines=eng_stats, option_less=bool(args.option_less))
        p.update(warmup_s=round(warm_s, 2), models={"nl2sql": f"duckdb-nsql-7B ({args.nl2sql_dtype})",
                                                    "explain_error": f"Llama-3.2-3B-Instruct ({args.explain_dtype})"},
                 new_tokens=args.new_tokens, explain_prompt_tokens_approx=args.explain_tokens,
                 tokenizer="byte-level (random-init)" if cpt == 1.0 else "model vocab",
                 explain_frac=args.explain_frac, engine=args.engine, data="synthetic prompts, random-init weights")
    return phases[0] if len(phases) == 1 else {"phases": phases}


def as_generate(route: str, body: dict) -> dict:
    """The /nl2sql or /explain_error request as the equivalent streaming ``/api/generate`` call (the
    same model, system and prompt strings the pipeline builds)."""
    from . import prompts

    if route == "nl2sql":
        return {"model": "duckdb-nsql", "system": prompts.nl2sql_system(body["table_schema"]),
                "prompt": body["question"], "options": body.get("options"), "stream": True}
    return {"model": "llama3.2", "system": prompts.EXPLAIN_SYSTEM,
            "prompt": prompts.explain_prompt(body["error_message"]), "options": body.get("options"), "stream": True}


def _phase(cl, args, qps: float, rng: random.Random, make_request) -> dict:
    """One fixed-rate load phase: a Poisson arrival schedule fixed up front, fired from a thread pool."""
    sched, t = [], 0.0
    while True:
        t += rng.expovariate(qps)
        if t >= args.duration:
            break
        sched.append((t, *make_request(len(sched))))
    results = []
    lock = threading.Lock()
    start = time.perf_counter()

    def fire(item):
        at, route, body = item
        delay = at - (time.perf_counter() - start)
        if delay > 0:
            time.sleep(delay)
        t1 = time.perf_counter()
        ttft = None
        try:
            if getattr(args, "stream", False):  # Ollama streaming API: time to the first response piece
                d = {}
                with cl.stream("POST", "/api/generate", json=as_generate(route, body)) as r:
                    ok = r.status_code == 200
                    for line in r.iter_lines():
                        if not line.strip():
                            continue
                        c = json.loads(line)
                        if ttft is None and not c.get("done"):  # first chunk = first token(s) out
                            ttft = time.perf_counter() - t1
                        if c.get("done"):
                            d = c
            else:
                r = cl.post("/" + route, json=body)
                ok = r.status_code == 200
                d = r.json() if ok else {}
        except Exception as e:  # noqa: BLE001 - counted as a failed request
            ok, d = False, {"error": repr(e)}
        lat = time.perf_counter() - t1
        with lock:
            results.append((route, ok, lat, int(d.get("eval_count", 0)), at, ttft))

    with ThreadPoolExecutor(max_workers=args.concurrency) as ex:
        list(ex.map(fire, sched))
    wall = time.perf_counter() - start
    out = {"metric": "co-serving output_tokens_per_sec @ fixed QPS", "qps_target": qps,
           "duration_s": args.duration, "wall_s": round(wall, 3),
           "requests": len(results), "failed": sum(1 for r in results if not r[1]),
           "achieved_qps": round(len(results) / wall, 3) if wall > 0 else None,
           "output_tokens_per_sec": round(sum(r[3] for r in results if r[1]) / wall, 2) if wall > 0 else None}
    for route in ("nl2sql", "explain_error"):
        lats = [r[2] for r in results if r[0] == route and r[1]]
        out[route] = {"n": len(lats), "p50_s": _pct(lats, 0.5), "p90_s": _pct(lats, 0.9), "p99_s": _pct(lats, 0.99),
                      "mean_s": round(statistics.fmean(lats), 4) if lats else None}
        ttfts = [r[5] for r in results if r[0] == route and r[1] and r[5] is not None]
        if ttfts:
            out[route].update(ttft_p50_s=_pct(ttfts, 0.5), ttft_p99_s=_pct(ttfts, 0.99))
    ref = {"nl2sql": 5.2381, "explain_error": 22.75}  # BASELINE.md p50s (other hardware, single requests)
    out["vs_baseline_p50_latency"] = {k: (round(ref[k] / out[k]["p50_s"], 2) if out[k]["p50_s"] else None)
                                      for k in ref}
    return out


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--qps", default="8", help="requests/s; a comma list runs one phase per rate")
    ap.add_argument("--duration", type=float, default=30.0, help="seconds of arrivals")
    ap.add_argument("--explain-frac", type=float, default=0.3)
    ap.add_argument("--explain-tokens", type=int, default=1024, help="approx. prompt tokens of the error text")
    ap.add_argument("--new-tokens", type=int, default=128)
    ap.add_argument("--nl2sql-dtype", default="fp8")
    ap.add_argument("--explain-dtype", default="bf16")
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--engine", default="hip", help="hip | fake (plumbing only)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--option-less", action="store_true",
                    help="requests carry no num_predict / ignore_eos (generate until EOS or the context window)")
    ap.add_argument("--stream", action="store_true",
                    help="send each request as a streaming /api/generate call and report time to first piece")
    print(json.dumps(run(ap.parse_args(argv))), flush=True)


if __name__ == "__main__":
    main()

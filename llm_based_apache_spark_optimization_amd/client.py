"""Ollama-compatible client API.

The reference's only model interface is ``ollama.generate(model=..., system=..., prompt=...)`` and it
reads ``.response`` (FastAPI/app.py:85-90,105-111; Flask/app.py:102-107,160-165;
Model_Evaluation_&_Comparision.py:23,114).  This module keeps that call shape::

    from llm_based_apache_spark_optimization_amd import client
    res = client.generate(model="duckdb-nsql", system=..., prompt=...)
    sql = res.response            # or res["response"]

and returns the timing fields Ollama reports (``eval_count``, ``eval_duration``, ``prompt_eval_*``,
``load_duration``, ``total_duration``).  Backends (``set_backend``):

* ``EngineService`` — in-process MI355X engines (one ``LLMEngine`` per model, continuous batching on a
  background thread so concurrent callers share decode steps);
* ``FakeBackend`` — deterministic canned outputs for tests (with fault injection);
* ``RemoteBackend`` — HTTP ``POST /api/generate`` on an Ollama-compatible server (this package's
  FastAPI app, or a real Ollama daemon);
* ``parallel.router.ReplicaRouter`` — data-parallel dispatch across engine replica processes.
"""
from __future__ import annotations

import dataclasses
import datetime as _dt
import json
import queue
import threading
import time
from typing import Callable, Dict, Iterator, Optional

import torch

from .engine.engine import SamplingParams


@dataclasses.dataclass
class GenerateResponse:
    model: str
    response: str
    done: bool = True
    done_reason: str = "stop"
    created_at: str = ""
    total_duration: int = 0
    load_duration: int = 0
    prompt_eval_count: int = 0
    prompt_eval_duration: int = 0
    eval_count: int = 0
    eval_duration: int = 0

    def __getitem__(self, k):
        return getattr(self, k)

    def get(self, k, default=None):
        return getattr(self, k, default)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @property
    def tokens_per_second(self) -> float:
        return self.eval_count / (self.eval_duration / 1e9) if self.eval_duration else 0.0


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).isoformat()


class Backend:
    def generate(self, model: str, prompt: str, system: str = "", options: Optional[dict] = None,
                 raw: bool = False) -> GenerateResponse:
        raise NotImplementedError

    def generate_stream(self, model: str, prompt: str, system: str = "", options: Optional[dict] = None,
                        raw: bool = False) -> Iterator[GenerateResponse]:
        """Ollama's streaming shape: chunks with ``done=False`` carrying response pieces, then one
        ``done=True`` chunk with an empty response and the timing fields.  Backends without incremental
        output send the whole answer as one piece."""
        r = self.generate(model, prompt, system, options, raw)
        yield GenerateResponse(model=model, response=r.response, done=False, done_reason="", created_at=r.created_at)
        yield dataclasses.replace(r, response="")

    def models(self) -> list:
        return []

    def health(self, deep: bool = False) -> dict:
        return {"ok": True}


# -------------------------------------------------------------------------------------- engines
class EngineUnavailable(RuntimeError):
    """The model's engine is down (its loop died and could not be restarted): the serving layer answers
    503 at once instead of letting requests wait for the timeout."""


def _fatal_device_error(e: BaseException) -> bool:
    """A GPU fault poisons the HIP context: the engine cannot be reset in this process."""
    from .engine.runner import TPCommError

    if isinstance(e, TPCommError):  # the lockstep TP group is out of sync: never step it again
        return True
    msg = str(e)
    return any(k in msg for k in ("HIP error", "hipError", "CUDA error", "illegal memory access",
                                  "device-side assert", "Memory access fault"))


class _EngineLoop:
    """Drives one LLMEngine from a background thread; callers block on their request's event.

    Failure handling: when a step raises, every queued / running request is failed at once
    (``LLMEngine.abort_all``) and the loop keeps serving -- up to ``max_errors`` failures inside
    ``error_window_s``.  A fatal device error, or too many failures, ends the loop; ``EngineService``
    then rebuilds the engine or answers ``EngineUnavailable``.

    ``every_error_fatal`` (the leader of a lockstep TP replica, parallel/lockstep.py): any step exception
    ends the loop, because a failure after a mirrored call left the followers inside collectives the leader
    never joins; ``on_fatal(e)`` then runs before any request is released (the TP leader exits, so the
    router re-dispatches its in-flight requests and terminates the followers)."""

    def __init__(self, engine, run_ahead: int = 16, max_errors: int = 3, error_window_s: float = 60.0,
                 every_error_fatal: bool = False, on_fatal: Optional[Callable[[BaseException], None]] = None):
        self.engine = engine
        self.max_errors, self.error_window_s = max_errors, error_window_s
        self.every_error_fatal, self.on_fatal = every_error_fatal, on_fatal
        self._errors: list = []
        self.restarts = 0
        engine.run_ahead = run_ahead  # serving: bound each decode run so arrivals are admitted promptly
        # each engine runs on its own HIP stream: co-served models overlap on the GPU, and one engine's
        # host syncs never wait for the other's queued kernels
        self.stream = None
        dev = getattr(getattr(engine, "runner", None), "device", None)
        if dev is not None and torch.device(dev).type == "cuda":
            self.stream = torch.cuda.Stream(device=dev)
            self.stream.wait_stream(torch.cuda.current_stream(dev))
        self._cv = threading.Condition()
        self._stop = False
        self._err: Optional[BaseException] = None
        self._t = threading.Thread(target=self._run, name=f"engine-{engine.name}", daemon=True)
        self._t.start()

    def submit(self, ids, params, stream: bool = False):
        if not self.alive():
            raise EngineUnavailable(f"engine {self.engine.name} is down: {self._err!r}")
        req = self.engine.add_request(ids, params, stream=stream)
        with self._cv:
            self._cv.notify()
        return req

    def _run(self):
        from .utils.metrics import REGISTRY

        while not self._stop:
            with self._cv:
                while not self._stop and not self.engine.has_work():
                    self._cv.wait(timeout=0.5)
            if self._stop:
                return
            try:
                if self.stream is not None:
                    with torch.cuda.stream(self.stream):
                        self.engine.step()
                else:
                    self.engine.step()
            except BaseException as e:  # noqa: BLE001 - surface to waiting callers
                REGISTRY.inc("lsa_engine_errors_total", 1, "engine step failures", model=self.engine.name)
                now = time.monotonic()
                self._errors = [t for t in self._errors if now - t < self.error_window_s] + [now]
                fatal = (self.every_error_fatal or _fatal_device_error(e)
                         or len(self._errors) > self.max_errors)
                if fatal:
                    self._err = e  # alive() turns false before any caller is released
                    if self.on_fatal is not None:
                        self.on_fatal(e)
                try:
                    self.engine.abort_all(repr(e))
                except BaseException:  # noqa: BLE001
                    self._err = e
                    fatal = True
                if fatal:
                    return
                self.restarts += 1  # the engine is empty and consistent again: keep serving

    def alive(self) -> bool:
        return self._t.is_alive() and self._err is None

    def close(self):
        self._stop = True
        with self._cv:
            self._cv.notify_all()


class EngineService(Backend):
    """Named in-process engines (built lazily through ``factory``) behind the Ollama call shape."""

    def __init__(self, factory: Callable[[str], object], defaults: Optional[dict] = None,
                 timeout_s: float = 300.0, max_rebuilds: int = 2, every_error_fatal: bool = False,
                 on_fatal: Optional[Callable[[BaseException], None]] = None):
        self._factory = factory
        self._loop_kw = dict(every_error_fatal=every_error_fatal, on_fatal=on_fatal)
        self._loops: Dict[str, _EngineLoop] = {}
        self._lock = threading.Lock()
        self.defaults = defaults or {}
        self.timeout_s = timeout_s
        self.max_rebuilds = max_rebuilds
        self.rebuilds: Dict[str, int] = {}
        self._build_err: Dict[str, BaseException] = {}

    def loop(self, model: str) -> _EngineLoop:
        """The model's engine loop, built on first use and rebuilt (at most ``max_rebuilds`` times) after
        its loop died; a model that cannot be (re)built raises ``EngineUnavailable``."""
        with self._lock:
            lp = self._loops.get(model)
            if lp is not None and lp.alive():
                return lp
            if lp is not None:  # dead loop: rebuild the engine once the old one is released
                if self.rebuilds.get(model, 0) >= self.max_rebuilds:
                    raise EngineUnavailable(f"engine {model} is down after {self.rebuilds[model]} rebuilds: "
                                            f"{lp._err!r}")
                self.rebuilds[model] = self.rebuilds.get(model, 0) + 1
                lp.close()
                del self._loops[model]
                lp = None
                if torch.cuda.is_available():
                    torch.cuda.empty_cache()
            try:
                self._loops[model] = _EngineLoop(self._factory(model), **self._loop_kw)
            except EngineUnavailable:
                raise
            except Exception as e:  # noqa: BLE001
                self._build_err[model] = e
                raise EngineUnavailable(f"engine {model} could not be built: {e!r}") from e
            return self._loops[model]

    def _submit(self, model, prompt, system, options, raw, stream=False):
        lp = self.loop(model)
        eng = lp.engine
        opts = dict(self.defaults)
        opts.update(options or {})
        # no num_predict (the reference's option-less calls): generate until EOS / the context window, as
        # Ollama does; the engine bounds it by num_ctx and its own max_new_cap
        params = SamplingParams.from_ollama_options(opts)
        ids = eng.encode(eng.render(prompt, system, raw))
        if params.num_ctx is not None:
            ids = eng.fit_context(ids, params.num_ctx, params.num_keep)
        return eng, lp.submit(ids, params, stream=stream)

    @staticmethod
    def _final(model, eng, req) -> GenerateResponse:
        r = eng.result(req)
        return GenerateResponse(model=model, response=r.text, done_reason=r.done_reason, created_at=_now(),
                                total_duration=r.total_duration_ns, load_duration=r.load_duration_ns,
                                prompt_eval_count=r.prompt_tokens, prompt_eval_duration=r.prompt_eval_duration_ns,
                                eval_count=r.eval_count, eval_duration=r.eval_duration_ns)

    def generate(self, model, prompt, system="", options=None, raw=False) -> GenerateResponse:
        eng, req = self._submit(model, prompt, system, options, raw)
        if not req.done.wait(self.timeout_s):
            raise TimeoutError(f"generation on {model} timed out after {self.timeout_s}s")
        if req.error:
            raise RuntimeError(f"engine {model} failed: {req.error}")
        return self._final(model, eng, req)

    def generate_stream(self, model, prompt, system="", options=None, raw=False) -> Iterator[GenerateResponse]:
        """Pieces of the answer as the engine's decode runs complete (every ``sync_every`` steps, or
        ``run_ahead`` steps for requests that ignore EOS), then the final chunk with the timings."""
        eng, req = self._submit(model, prompt, system, options, raw, stream=True)
        try:
            for piece in eng.stream_text(req, timeout_s=self.timeout_s):
                yield GenerateResponse(model=model, response=piece, done=False, done_reason="", created_at=_now())
        except queue.Empty:
            raise TimeoutError(f"generation on {model} timed out after {self.timeout_s}s") from None
        except RuntimeError as e:
            raise RuntimeError(f"engine {model} failed: {e}") from None
        yield dataclasses.replace(self._final(model, eng, req), response="")

    def models(self) -> list:
        return sorted(self._loops)

    def health(self, deep: bool = False) -> dict:
        return {"ok": all(lp.alive() for lp in self._loops.values()),
                "engines": {m: {"alive": lp.alive(), "running": lp.engine.sched.num_running,
                                "waiting": lp.engine.sched.num_waiting, "kv_usage": lp.engine.sched.kv_usage,
                                "restarts": lp.restarts, "rebuilds": self.rebuilds.get(m, 0),
                                **lp.engine.stats} for m, lp in self._loops.items()}}


# -------------------------------------------------------------------------------------- fake
class FakeBackend(Backend):
    """Deterministic stand-in for tests: NL->SQL returns ``sql_for(prompt)``, explain returns a fixed
    analysis.  ``fail_next`` injects an exception (failure-path tests)."""

    def __init__(self, sql: Optional[Callable[[str, str], str]] = None, explanation: str = ""):
        self.sql = sql or (lambda prompt, system: "SELECT * FROM temp_view LIMIT 10;")
        self.explanation = explanation or ("The query references a column that does not exist in temp_view. "
                                           "Check the column names in the table schema and correct the query.")
        self.calls = []
        self.fail_next: Optional[BaseException] = None
        self._lock = threading.Lock()

    def generate(self, model, prompt, system="", options=None, raw=False) -> GenerateResponse:
        with self._lock:
            self.calls.append({"model": model, "prompt": prompt, "system": system, "options": options})
            if self.fail_next is not None:
                e, self.fail_next = self.fail_next, None
                raise e
        t0 = time.perf_counter()
        if options and options.get("fake_delay"):
            time.sleep(float(options["fake_delay"]))
        text = self.explanation if "Spark error" in prompt or "troubleshoot" in system else self.sql(prompt, system)
        dt = int((time.perf_counter() - t0) * 1e9)
        return GenerateResponse(model=model, response=text, created_at=_now(), total_duration=dt,
                                eval_count=len(text.split()), eval_duration=dt, prompt_eval_count=len(prompt.split()))

    def models(self):
        return ["duckdb-nsql", "llama3.2", "mistral"]


# -------------------------------------------------------------------------------------- remote
class RemoteBackend(Backend):
    def __init__(self, url: str = "http://127.0.0.1:8000", timeout_s: float = 300.0):
        self.url = url.rstrip("/")
        self.timeout_s = timeout_s

    def generate(self, model, prompt, system="", options=None, raw=False) -> GenerateResponse:
        import urllib.request

        body = json.dumps({"model": model, "prompt": prompt, "system": system, "options": options or {},
                           "stream": False, "raw": raw}).encode()
        req = urllib.request.Request(self.url + "/api/generate", data=body, headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=self.timeout_s) as f:
            d = json.loads(f.read())
        fields = {f.name for f in dataclasses.fields(GenerateResponse)}
        return GenerateResponse(**{k: v for k, v in d.items() if k in fields})


# -------------------------------------------------------------------------------------- module API
_backend: Optional[Backend] = None
_blk = threading.Lock()


def set_backend(b: Backend) -> None:
    global _backend
    with _blk:
        _backend = b


def get_backend() -> Backend:
    global _backend
    with _blk:
        if _backend is None:
            from .serving.service import backend_from_settings
            from .config import Settings

            _backend = backend_from_settings(Settings())
        return _backend


def generate(model: str, prompt: str = "", system: str = "", options: Optional[dict] = None, raw: bool = False,
             **_ignored) -> GenerateResponse:
    """Drop-in for ``ollama.generate(model=, system=, prompt=)``."""
    return get_backend().generate(model, prompt, system, options, raw)

"""LLMEngine: continuous-batching text generation over a ModelRunner.

The request lifecycle mirrors what the reference gets from the Ollama daemon behind
``ollama.generate(model=, system=, prompt=)`` (FastAPI/app.py:85-90,105-109; Flask/app.py:102-107,
160-164; Model_Evaluation_&_Comparision.py:23,114): template -> tokenize -> prefill -> decode loop ->
detokenize, with the timing fields Ollama reports (and the reference ignored).

Scheduling is native (``runtime/_lsa_runtime.Scheduler``): FCFS admission into fixed decode slots.  KV is
reserved lazily: admission takes the prompt plus one 64-token block, each decode run first grows the running
tables to the context the run will reach, and when the arena is exhausted the youngest running request is
preempted (blocks and slot released, re-queued first with its generated tokens folded into its prompt and
re-prefilled on re-admission).  Each engine iteration prefills newly admitted
requests (packed, one launch sequence) and then replays the captured decode graph for
``sync_every`` steps before reading the finished flags back — the host touches the GPU once per
``sync_every`` tokens, not once per token.
"""
from __future__ import annotations

import dataclasses
import itertools
import queue
import threading
import time
from typing import Callable, Iterator, Optional, Sequence

import torch

from ..models.templates import STOP_STRINGS, apply_stops, render
from ..models.tokenizer import tokenizer_for
from ..ops.reference import pack_seed
from ..runtime import native
from ..utils import tracing
from ..utils.metrics import REGISTRY, TOKEN_BUCKETS
from .runner import BLOCK, ModelRunner


UNLIMITED = 1 << 30  # max_tokens of a request without num_predict: EOS / context window end it


@dataclasses.dataclass
class SamplingParams:
    """Ollama-compatible options (temperature 0 = greedy, as the benchmark configs require)."""

    max_tokens: int = 128
    temperature: float = 0.0
    top_k: int = 40
    top_p: float = 0.9
    seed: Optional[int] = None
    ignore_eos: bool = False
    stop: tuple = ()
    # llama.cpp/Ollama repetition penalty over the last repeat_last_n (<= 64) context tokens.  1.0 = off
    # unless a request sets it (Ollama's own default is 1.1; the benchmark configs are plain greedy)
    repeat_penalty: float = 1.0
    repeat_last_n: int = 64
    num_ctx: Optional[int] = None     # Ollama context window (prompt + generated tokens); None = model's
    num_keep: int = 4

    @property
    def needs_sampler(self) -> bool:
        """Rows that need the sampling path (draw and/or penalty) rather than the argmax-only graph."""
        return self.temperature > 0 or self.repeat_penalty != 1.0

    @staticmethod
    def from_ollama_options(opts: Optional[dict], default_max: int = UNLIMITED) -> "SamplingParams":
        """Ollama option dict -> params.  ``num_predict`` absent, None or negative = Ollama's default: generate
        until EOS or the context window (``LLMEngine.add_request`` bounds it by num_ctx / max_new_cap)."""
        opts = opts or {}
        n = opts.get("num_predict", default_max)
        if n is None or int(n) < 0:
            n = default_max if default_max is not None and default_max >= 0 else UNLIMITED
        stop = opts.get("stop") or ()
        # ignore_eos: benchmark extension (fixed-length outputs from random-init weights), not an Ollama option
        return SamplingParams(max_tokens=int(n), temperature=float(opts.get("temperature", 0.0)),
                              top_k=int(opts.get("top_k", 40)), top_p=float(opts.get("top_p", 0.9)),
                              seed=opts.get("seed"), stop=tuple(stop), ignore_eos=bool(opts.get("ignore_eos", False)),
                              repeat_penalty=float(opts.get("repeat_penalty", 1.0)),
                              repeat_last_n=int(opts.get("repeat_last_n", 64)),
                              num_ctx=int(opts["num_ctx"]) if opts.get("num_ctx") else None,
                              num_keep=int(opts.get("num_keep", 4)))


@dataclasses.dataclass
class Request:
    rid: int
    prompt_ids: list
    params: SamplingParams
    arrival: float
    admitted: float = 0.0
    first_token: float = 0.0
    finished_at: float = 0.0
    output_ids: list = dataclasses.field(default_factory=list)
    done: threading.Event = dataclasses.field(default_factory=threading.Event)
    slot: int = -1
    gen_host: int = 0  # generated-token count as of the last device sync
    prefilled: int = 0  # prompt tokens already in the KV cache (chunked prefill in progress when < len)
    error: Optional[str] = None
    # streaming: ("tokens", ids-so-far) after every host sync that saw new tokens, then ("done", None)
    stream: Optional[queue.Queue] = None
    streamed: int = 0
    # tokens generated before a preemption (lazy KV growth ran the arena dry): the current incarnation's prompt is
    # prompt_ids + resumed and its params.max_tokens the remaining budget
    resumed: list = dataclasses.field(default_factory=list)
    preemptions: int = 0

    @property
    def ctx_ids(self) -> list:
        """Tokens the current incarnation prefills: the prompt plus anything generated before a preemption."""
        return self.prompt_ids + self.resumed if self.resumed else self.prompt_ids


@dataclasses.dataclass
class GenerationResult:
    text: str
    token_ids: list
    prompt_tokens: int
    eval_count: int
    total_duration_ns: int
    load_duration_ns: int
    prompt_eval_duration_ns: int
    eval_duration_ns: int
    done_reason: str


class LLMEngine:
    def __init__(self, runner: ModelRunner, tokenizer=None, max_prefill_tokens: int = 16384, sync_every: int = 8,
                 name: Optional[str] = None, prefill_chunk: Optional[int] = None, kv_reserve_tokens: int = BLOCK):
        self.runner = runner
        self.spec = runner.spec
        self.name = name or self.spec.name
        self.tok = tokenizer or tokenizer_for(self.spec)
        tok_eos = [e for e in getattr(self.tok, "eos_ids", ()) if 0 <= e < self.spec.vocab_size]
        if tok_eos and sorted(tok_eos) != sorted(runner.eos_list):
            runner.set_eos(sorted(set(tok_eos) | set(e for e in runner.eos_list if e >= 0)))
        # kv_reserve_tokens: generated tokens reserved at admission (< 0: prompt + max_new up front, no growth)
        self.sched = native.Scheduler(runner.num_kv_blocks, BLOCK, runner.max_slots, max_prefill_tokens,
                                      runner.max_blocks, kv_reserve_tokens)
        # set by a preemption: no admissions while requests run and fewer than _admit_hold_blocks KV blocks are free
        # (the preempted request's re-admission plus one block of growth per running request), so the preempted
        # request is not re-admitted at once and evicted again by the same growth
        self._admit_hold = False
        self._admit_hold_blocks = 0
        self.sync_every = sync_every
        # decode steps per iteration when every running request ignores EOS: None = run to the first
        # length limit (offline batches); a server sets a bound so new arrivals are admitted promptly
        self.run_ahead: Optional[int] = None
        self.max_prefill_tokens = max_prefill_tokens
        # chunked-prefill interleave (serving): at most this many prompt tokens are prefilled per engine
        # iteration, so a long prompt (a 2k-token Spark error for /explain_error) is spread over several
        # iterations with decode runs of the already-running requests in between instead of stalling them
        # for its whole prefill.  None = prefill every admitted prompt at once (offline batches, bench.py).
        self.prefill_chunk = prefill_chunk
        self._prefilling: list = []  # admitted requests whose prompt is not fully in the KV cache yet
        self._ids = itertools.count(1)
        self._reqs: dict[int, Request] = {}
        self._lock = threading.RLock()
        self._slot_owner: dict[int, int] = {}
        self.load_time_s = 0.0
        self.stats = {"requests": 0, "prompt_tokens": 0, "generated_tokens": 0, "decode_steps": 0,
                      "prefill_s": 0.0, "decode_s": 0.0, "decode_device_s": 0.0, "aborted": 0, "preempted": 0,
                      "kv_grown_blocks": 0, "peak_running": 0}
        # per-decode-run device timing (hipEvents around the graph replays, read after the host sync the
        # run ends with anyway): lsa_decode_step_device_seconds{model} = GPU time per token step
        self.device_timing = runner.on_gpu

    # -------------------------------------------------------------------------------- prompts
    def render(self, prompt: str, system: str = "", raw: bool = False) -> str:
        return prompt if raw else render(self.spec.template, prompt, system)

    @staticmethod
    def fit_context(ids: Sequence[int], num_ctx: int, num_keep: int = 4) -> list[int]:
        """Ollama's ``num_ctx`` window: a prompt of more than num_ctx - 1 tokens keeps its
        first ``num_keep`` tokens (BOS + template head) and its tail, dropping the middle, so at least one
        token can be generated.  Generation then stops at the window (``add_request`` caps max_tokens);
        Ollama would shift the context instead."""
        limit = max(1, int(num_ctx) - 1)
        ids = list(ids)
        if len(ids) <= limit:
            return ids
        keep = max(0, min(int(num_keep), limit - 1))
        return ids[:keep] + ids[len(ids) - (limit - keep):]

    def encode(self, text: str) -> list[int]:
        ids = self.tok.encode(text, add_bos=True)
        limit = self.runner.max_model_len - 1
        return ids[-limit:] if len(ids) > limit else ids

    # -------------------------------------------------------------------------------- request API
    def add_request(self, prompt_ids: Sequence[int], params: SamplingParams, stream: bool = False) -> Request:
        window = self.runner.max_model_len if params.num_ctx is None else min(self.runner.max_model_len,
                                                                               int(params.num_ctx))
        room = window - len(prompt_ids)
        if room < 1:
            raise ValueError("prompt longer than the model context")
        p = dataclasses.replace(params, max_tokens=max(1, min(params.max_tokens, room, self.runner.max_new_cap)))
        req = Request(next(self._ids), list(map(int, prompt_ids)), p, time.perf_counter(),
                      stream=queue.Queue() if stream else None)
        with self._lock:
            self.sched.add(req.rid, len(req.prompt_ids), p.max_tokens)
            self._reqs[req.rid] = req
        return req

    def has_work(self) -> bool:
        return self.sched.num_waiting > 0 or self.sched.num_running > 0 or bool(self._prefilling)

    def step(self) -> list[Request]:
        """One engine iteration: admit + prefill new requests (at most ``prefill_chunk`` prompt tokens when
        set), run decode steps over the requests whose prompt is complete, retire finished ones."""
        r = self.runner
        with self._lock:
            # after a preemption, admit nothing while requests still run: the preempted one would otherwise be
            # re-admitted at once and evicted again by the same growth
            if self._admit_hold and (self.sched.num_running == 0 or self.sched.free_blocks >= self._admit_hold_blocks):
                self._admit_hold = False
            admitted = [] if self._admit_hold else self.sched.admit()
            self.stats["peak_running"] = max(self.stats["peak_running"], self.sched.num_running)
            t0 = time.perf_counter()
            entries = []
            for rid in admitted:
                req = self._reqs[rid]
                slot = self.sched.slot(rid)
                req.slot = slot
                req.admitted = req.admitted or t0
                self._slot_owner[slot] = rid
                sp = req.params
                # a re-admitted (preempted) request continues its random stream where it stopped: the sampler draws
                # token g from the stream keyed by the seed at counter g + offset (ops/reference.py draw_seed,
                # sampling.hip), and this incarnation's g restarts at 0 after len(resumed) tokens
                seed = pack_seed(sp.seed if sp.seed is not None else (rid * 7919 + 17), len(req.resumed))
                entries.append(dict(slot=slot, blocks=self.sched.block_table(rid), limit=sp.max_tokens,
                                    temperature=sp.temperature, top_k=sp.top_k, top_p=sp.top_p, seed=seed,
                                    eos_on=not sp.ignore_eos, repeat_penalty=sp.repeat_penalty,
                                    repeat_last_n=sp.repeat_last_n, prompt_ids=req.ctx_ids,
                                    defer_table=self.prefill_chunk is not None))
                self._prefilling.append(req)
            r.set_slots(entries)  # one batched host -> device transfer for every admitted request
            if self._prefilling:
                done_now = self._prefill_some()
                t1 = time.perf_counter()
                for q in done_now:
                    q.first_token = q.first_token or t1
                    q.gen_host = 1
                    if q.stream is not None:  # the prefill's token goes out now (one sync, streaming only)
                        q.streamed = len(q.resumed) + 1
                        q.stream.put(("tokens", q.resumed + r.tokens_of(q.slot, 1)))
                self.stats["prefill_s"] += t1 - t0
            pending = {q.rid for q in self._prefilling}
            running = [rid for rid in self.sched.running() if rid not in pending]
            if not running:
                return []
            sample = any(self._reqs[rid].params.needs_sampler for rid in running)
            # steps until the earliest request can hit its length limit; with EOS possible, at most
            # sync_every steps between host checks
            reqs = [self._reqs[rid] for rid in running]
            remaining = min(q.params.max_tokens - q.gen_host for q in reqs)
            if remaining <= 0:
                n_steps = 0  # a request finished with its prefill token (max_tokens 1): retire it first
            elif all(q.params.ignore_eos for q in reqs):
                n_steps = remaining if self.run_ahead is None else min(self.run_ahead, remaining)
            else:
                n_steps = min(self.sync_every, remaining)
            if n_steps:
                reqs = self._grow_kv(reqs, n_steps)  # lazy KV: grow the tables for this run, preempting if needed
                running = [q.rid for q in reqs]
                if not reqs:
                    return []
            B = r.bucket(self.sched.highest_slot + 1)
            # host-side bound on every row's context during the run (selects the decode graph's split plan)
            max_ctx = max(len(q.ctx_ids) + min(q.gen_host + n_steps, q.params.max_tokens) for q in reqs) + 1
        # the decode run needs no scheduler state: new requests may be added meanwhile
        t0 = time.perf_counter()
        ev = None
        if n_steps:
            if self.device_timing:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            r.decode(B, n_steps, sample, max_ctx=max_ctx)
            if ev is not None:
                ev[1].record()
        fin, gl, _ = r.read_rows([q.slot for q in reqs])
        with self._lock:
            self.stats["decode_s"] += time.perf_counter() - t0
            self.stats["decode_steps"] += n_steps
            if ev is not None:
                dev_s = ev[0].elapsed_time(ev[1]) / 1e3  # both recorded before read_rows' sync
                self.stats["decode_device_s"] += dev_s
                REGISTRY.observe("lsa_decode_step_device_seconds", dev_s / n_steps, "GPU time per decode step",
                                 buckets=TOKEN_BUCKETS, model=self.name, batch=str(B))
            done = []
            now = time.perf_counter()
            # generated tokens of every finished row in one device -> host transfer
            fin_rows = [(self._reqs[rid].slot, min(int(gl[i]), self._reqs[rid].params.max_tokens))
                        for i, rid in enumerate(running) if int(fin[i])]
            fin_toks = dict(zip([s for s, _ in fin_rows], r.tokens_of_many([s for s, _ in fin_rows],
                                                                           [n for _, n in fin_rows])))
            for i, rid in enumerate(running):
                self._reqs[rid].gen_host = int(gl[i])
                q = self._reqs[rid]
                if q.stream is not None and not int(fin[i]):
                    n = min(int(gl[i]), q.params.max_tokens)
                    if len(q.resumed) + n > q.streamed:  # the rows are host-visible after read_rows' sync
                        q.streamed = len(q.resumed) + n
                        q.stream.put(("tokens", q.resumed + r.tokens_of(q.slot, n)))
                if int(fin[i]):
                    req = self._reqs.pop(rid)
                    req.output_ids = req.resumed + fin_toks[req.slot]
                    n = len(req.output_ids)
                    self._admit_hold = False
                    req.finished_at = now
                    r.release_slot(req.slot)
                    self._slot_owner.pop(req.slot, None)
                    self.sched.finish(rid)
                    self.stats["generated_tokens"] += n
                    self.stats["requests"] += 1
                    self._trace_done(req, n)
                    req.done.set()
                    if req.stream is not None:
                        req.stream.put(("done", None))
                    done.append(req)
            return done

    def _grow_kv(self, reqs: list, n_steps: int) -> list:
        """Lazy KV reservation: before a decode run of ``n_steps`` every running request must own the blocks of
        every cache position the run writes (the context after the run, less the last generated token, which is
        never written).  Requests grow oldest admission first; when the arena runs dry the youngest running
        request is preempted (possibly the one growing).  Returns the requests that stay in the run; the device
        block tables of the grown ones are updated in one batched transfer."""
        need = {q.rid: len(q.ctx_ids) + min(q.gen_host - 1 + n_steps, q.params.max_tokens - 1) for q in reqs}
        order = self.sched.youngest_first()
        alive = set(need)
        grown = {}
        for rid in reversed(order):  # oldest first
            if rid not in alive:
                continue
            while True:
                got = self.sched.grow(rid, need[rid])
                if got >= 0:
                    if got > 0:
                        grown[rid] = got
                    break
                victim = next(v for v in order if v in alive)
                self._preempt(self._reqs[victim])
                alive.discard(victim)
                grown.pop(victim, None)
                if victim == rid:
                    break
        if grown:
            self.stats["kv_grown_blocks"] += sum(grown.values())
            self.runner.extend_tables([(self._reqs[rid].slot, self.sched.block_table(rid)) for rid in grown])
        return [q for q in reqs if q.rid in alive]

    def _preempt(self, q: Request) -> None:
        """Release a running request's slot and KV blocks and re-queue it first; its generated tokens become part
        of the prompt it re-prefills (recompute), its budget shrinks by as many."""
        n = min(q.gen_host, q.params.max_tokens)
        toks = self.runner.tokens_of(q.slot, n) if n else []
        q.resumed = q.resumed + toks
        q.params = dataclasses.replace(q.params, max_tokens=q.params.max_tokens - n)
        self.runner.release_slot(q.slot)
        self._slot_owner.pop(q.slot, None)
        self.sched.preempt(q.rid, len(q.ctx_ids), q.params.max_tokens)
        q.slot, q.gen_host, q.prefilled = -1, 0, 0
        q.preemptions += 1
        self.stats["preempted"] += 1
        reserve = self.sched.reserve_tokens
        gen = q.params.max_tokens if reserve < 0 else min(q.params.max_tokens, reserve)
        self._admit_hold = True
        self._admit_hold_blocks = -(-(len(q.ctx_ids) + gen) // BLOCK) + self.sched.num_running

    def _trace_done(self, req: Request, n: int) -> None:
        """Engine spans of a finished request (queue -> prefill -> decode), fed to lsa_stage_seconds and,
        with LSA_TRACE=1, to the JSONL trace (SURVEY.md §5 tracing)."""
        rid = f"{self.name}:{req.rid}"
        tracing.record("engine_queue", req.admitted - req.arrival, rid, model=self.name)
        tracing.record("engine_prefill", req.first_token - req.admitted, rid, model=self.name,
                       prompt_tokens=len(req.prompt_ids))
        tracing.record("engine_decode", req.finished_at - req.first_token, rid, model=self.name, tokens=n)

    def abort_all(self, reason: str) -> list:
        """Fail every queued and running request (engine recovery after a step raised): their callers are
        released with ``error`` set, slots and KV blocks are returned, the engine is empty again."""
        with self._lock:
            out = []
            now = time.perf_counter()
            for rid, req in list(self._reqs.items()):
                req.error = reason
                req.finished_at = now
                if req.slot >= 0:
                    try:
                        self.runner.release_slot(req.slot)
                    except Exception:  # noqa: BLE001 - a faulted device: the engine is rebuilt anyway
                        pass
                self.sched.finish(rid)
                req.done.set()
                if req.stream is not None:
                    req.stream.put(("done", None))
                out.append(req)
            self._reqs.clear()
            self._slot_owner.clear()
            self._prefilling.clear()
            self.stats["aborted"] += len(out)
            return out

    def _prefill_some(self) -> list:
        """Prefill the admitted-but-incomplete prompts FCFS within this iteration's token budget; returns the
        requests whose prompt completed (their first token is committed)."""
        budget = self.prefill_chunk if self.prefill_chunk else None
        final, partial, done = [], [], []
        any_sample = False
        for q in list(self._prefilling):
            ids = q.ctx_ids
            rest = len(ids) - q.prefilled
            take = rest if budget is None else min(rest, budget)
            if take <= 0:
                break
            seg = (q.slot, ids[q.prefilled:q.prefilled + take], q.prefilled)
            q.prefilled += take
            if q.prefilled == len(ids):
                final.append(seg)
                done.append(q)
                any_sample |= q.params.needs_sampler
                self._prefilling.remove(q)
            else:
                partial.append(seg)
            self.stats["prompt_tokens"] += take
            if budget is not None:
                budget -= take
                if budget <= 0:
                    break
        if partial:  # KV only (no token commit); chunks of different requests pack into one launch sequence
            self.runner.prefill_chunk(partial)
        if final:
            self._prefill_packed(final, any_sample)
        return done

    def _prefill_packed(self, seqs, any_sample: bool) -> None:
        """Prefill in chunks of at most max_prefill_tokens tokens (long prompts split across calls)."""
        r = self.runner
        batch, tokens = [], 0
        for slot, ids, p0 in seqs:
            if len(ids) > self.max_prefill_tokens:  # chunked prefill of one long prompt
                if batch:
                    r.prefill(batch, any_sample)
                    batch, tokens = [], 0
                c = self.max_prefill_tokens
                for s in range(0, len(ids) - c, c):
                    r.prefill_chunk([(slot, ids[s:s + c], p0 + s)])
                s = ((len(ids) - 1) // c) * c
                r.prefill([(slot, ids[s:], p0 + s)], any_sample)
                continue
            if tokens + len(ids) > self.max_prefill_tokens and batch:
                r.prefill(batch, any_sample)
                batch, tokens = [], 0
            batch.append((slot, ids, p0))
            tokens += len(ids)
        if batch:
            r.prefill(batch, any_sample)

    def run_until_done(self, reqs: Sequence[Request]) -> None:
        while not all(q.done.is_set() for q in reqs):
            self.step()

    # -------------------------------------------------------------------------------- one-shot API
    def result(self, req: Request, template: Optional[str] = None) -> GenerationResult:
        t0 = time.perf_counter()
        text = self.tok.decode(req.output_ids)
        text = apply_stops(text, template or self.spec.template, req.params.stop)
        tracing.record("engine_detok", time.perf_counter() - t0, f"{self.name}:{req.rid}", model=self.name)
        ns = lambda s: int(max(0.0, s) * 1e9)  # noqa: E731
        ended_eos = bool(req.output_ids) and req.output_ids[-1] in self.runner.eos_list and not req.params.ignore_eos
        return GenerationResult(
            text=text, token_ids=req.output_ids, prompt_tokens=len(req.prompt_ids), eval_count=len(req.output_ids),
            total_duration_ns=ns(req.finished_at - req.arrival), load_duration_ns=ns(self.load_time_s),
            prompt_eval_duration_ns=ns(req.first_token - req.admitted),
            eval_duration_ns=ns(req.finished_at - req.first_token), done_reason="stop" if ended_eos else "length")

    def text_of(self, token_ids: Sequence[int], req: Request) -> str:
        """The response text of ``token_ids`` exactly as ``result`` builds it (stop strings applied)."""
        return apply_stops(self.tok.decode(list(token_ids)), self.spec.template, req.params.stop)

    def stream_text(self, req: Request, timeout_s: Optional[float] = None) -> Iterator[str]:
        """Text pieces of a request added with ``stream=True``, one per host sync that revealed tokens.
        The pieces concatenate to ``result(req).text``: a trailing incomplete UTF-8 sequence and any
        tail that could still grow into a stop string are held back until later tokens settle them, and
        nothing past a stop string is sent."""
        assert req.stream is not None, "add_request(..., stream=True)"
        stops = tuple(STOP_STRINGS.get(self.spec.template, ())) + tuple(req.params.stop)
        sent = 0
        while True:
            kind, toks = req.stream.get(timeout=timeout_s)
            if kind == "done":
                break
            raw = self.tok.decode(list(toks))
            text = self.text_of(toks, req)
            if len(text) < len(raw):  # a stop string appeared: only its prefix is ever sent
                safe = len(text)
            else:
                safe = len(text.rstrip("\ufffd"))
                hold = 0  # the longest tail that is a proper prefix of a stop string
                for st in stops:
                    for k in range(min(len(st) - 1, safe), hold, -1):
                        if text[safe - k:safe] == st[:k]:
                            hold = k
                            break
                safe -= hold
            # one piece per snapshot, empty while no new text is settled (tokens that decode to nothing,
            # held-back tails): the client sees progress at every sync, as with Ollama's per-token chunks
            piece = text[sent:safe] if safe > sent else ""
            sent = max(sent, safe)
            yield piece
        if req.error:
            raise RuntimeError(req.error)
        final = self.result(req).text
        if len(final) > sent:
            yield final[sent:]

    def generate(self, prompts: Sequence, params: Optional[SamplingParams] = None, system: str = "",
                 raw: bool = False) -> list[GenerationResult]:
        """Batch generate. ``prompts``: strings (templated + tokenized) or token-id lists."""
        params = params or SamplingParams()
        reqs = []
        for p in prompts:
            ids = self.encode(self.render(p, system, raw)) if isinstance(p, str) else list(p)
            if params.num_ctx is not None:
                ids = self.fit_context(ids, params.num_ctx, params.num_keep)
            reqs.append(self.add_request(ids, params))
        self.run_until_done(reqs)
        return [self.result(q) for q in reqs]

    def generate_text(self, prompt: str, system: str = "", params: Optional[SamplingParams] = None,
                      on_token: Optional[Callable[[str], None]] = None) -> GenerationResult:
        res = self.generate([prompt], params, system)[0]
        if on_token is not None:
            on_token(res.text)
        return res

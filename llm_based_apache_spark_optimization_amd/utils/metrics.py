"""Minimal Prometheus text-format metrics registry (counters, gauges, latency histograms).

Replaces the reference's emoji ``print`` observability (FastAPI/app.py:48,51; Flask/app.py:43,45):
request counts per route/outcome, end-to-end and per-stage latencies (queue, tokenize, prefill,
decode, SQL, history), generated tokens, TTFT / TPOT and engine gauges (running, waiting, KV usage).
"""
from __future__ import annotations

import bisect
import threading
from collections import defaultdict

_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0, 120.0)
# per-token latencies (TPOT, device step time) and generation rates need their own scales
TOKEN_BUCKETS = (0.0005, 0.001, 0.0015, 0.002, 0.003, 0.004, 0.005, 0.0075, 0.01, 0.02, 0.05, 0.1, 0.25)
RATE_BUCKETS = (10, 25, 50, 100, 200, 300, 400, 500, 750, 1000, 2000, 5000)


def _lbl(labels: dict) -> str:
    if not labels:
        return ""
    return "{" + ",".join(f'{k}="{str(v)}"' for k, v in sorted(labels.items())) + "}"


class Registry:
    def __init__(self):
        self._lock = threading.Lock()
        self._counters = defaultdict(float)
        self._gauges = {}
        self._hist = {}
        self._help = {}

    def inc(self, name: str, value: float = 1.0, help: str = "", **labels) -> None:
        with self._lock:
            self._counters[(name, _lbl(labels))] += value
            self._help.setdefault(name, (help, "counter"))

    def set(self, name: str, value: float, help: str = "", **labels) -> None:
        with self._lock:
            self._gauges[(name, _lbl(labels))] = value
            self._help.setdefault(name, (help, "gauge"))

    def observe(self, name: str, value: float, help: str = "", buckets: tuple = _BUCKETS, **labels) -> None:
        with self._lock:
            key = (name, _lbl(labels))
            h = self._hist.get(key)
            if h is None:
                h = self._hist[key] = [[0] * (len(buckets) + 1), 0.0, 0, buckets]
            b = h[3]
            h[0][bisect.bisect_left(b, value)] += 1
            h[1] += value
            h[2] += 1
            self._help.setdefault(name, (help, "histogram"))

    def quantile(self, name: str, q: float, **labels) -> float:
        """Approximate quantile from the histogram buckets (upper bound of the bucket)."""
        h = self._hist.get((name, _lbl(labels)))
        if not h or not h[2]:
            return 0.0
        target, acc = q * h[2], 0
        for i, c in enumerate(h[0]):
            acc += c
            if acc >= target:
                return h[3][i] if i < len(h[3]) else float("inf")
        return float("inf")

    def count(self, name: str, **labels) -> int:
        h = self._hist.get((name, _lbl(labels)))
        return h[2] if h else 0

    def value(self, name: str, **labels) -> float:
        key = (name, _lbl(labels))
        return self._counters.get(key, self._gauges.get(key, 0.0))

    def render(self) -> str:
        out = []
        with self._lock:
            seen = set()
            for (name, lbl), v in sorted(self._counters.items()):
                if name not in seen:
                    out.append(f"# HELP {name} {self._help[name][0]}\n# TYPE {name} counter")
                    seen.add(name)
                out.append(f"{name}{lbl} {v}")
            for (name, lbl), v in sorted(self._gauges.items()):
                if name not in seen:
                    out.append(f"# HELP {name} {self._help[name][0]}\n# TYPE {name} gauge")
                    seen.add(name)
                out.append(f"{name}{lbl} {v}")
            for (name, lbl), (counts, s, n, bks) in sorted(self._hist.items()):
                if name not in seen:
                    out.append(f"# HELP {name} {self._help[name][0]}\n# TYPE {name} histogram")
                    seen.add(name)
                acc = 0
                base = lbl[1:-1] if lbl else ""
                for b, c in zip(bks, counts):
                    acc += c
                    sep = "," if base else ""
                    out.append(f'{name}_bucket{{{base}{sep}le="{b}"}} {acc}')
                sep = "," if base else ""
                out.append(f'{name}_bucket{{{base}{sep}le="+Inf"}} {n}')
                out.append(f"{name}_sum{lbl} {s}")
                out.append(f"{name}_count{lbl} {n}")
        return "\n".join(out) + "\n"


REGISTRY = Registry()


def record_generation(res, route: str = "") -> None:
    """Per-request generation metrics from an Ollama-style response (``client.GenerateResponse``; durations
    in ns): TTFT = arrival -> first token (total - eval duration), TPOT = decode time per token after the
    first, decode rate, token counters.  Fed at the serving layer, so in-process engines, DP replica
    routers and remote backends are all measured the same way."""
    model = getattr(res, "model", "") or "unknown"
    n = int(getattr(res, "eval_count", 0) or 0)
    tot, ev = int(getattr(res, "total_duration", 0) or 0), int(getattr(res, "eval_duration", 0) or 0)
    lbl = {"model": model} if not route else {"model": model, "route": route}
    REGISTRY.inc("lsa_generated_tokens_total", n, "tokens generated", **lbl)
    REGISTRY.inc("lsa_prompt_tokens_total", int(getattr(res, "prompt_eval_count", 0) or 0), "prompt tokens", **lbl)
    if tot > 0:
        REGISTRY.observe("lsa_ttft_seconds", max(0, tot - ev) / 1e9, "time to first token", **lbl)
    if n > 1 and ev > 0:
        REGISTRY.observe("lsa_tpot_seconds", ev / 1e9 / (n - 1), "time per output token after the first",
                         buckets=TOKEN_BUCKETS, **lbl)
        REGISTRY.observe("lsa_decode_tokens_per_second", (n - 1) / (ev / 1e9), "per-request decode rate",
                         buckets=RATE_BUCKETS, **lbl)

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

    def observe(self, name: str, value: float, help: str = "", **labels) -> None:
        with self._lock:
            key = (name, _lbl(labels))
            h = self._hist.get(key)
            if h is None:
                h = self._hist[key] = [[0] * (len(_BUCKETS) + 1), 0.0, 0]
            h[0][bisect.bisect_left(_BUCKETS, value)] += 1
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
                return _BUCKETS[i] if i < len(_BUCKETS) else float("inf")
        return float("inf")

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
            for (name, lbl), (counts, s, n) in sorted(self._hist.items()):
                if name not in seen:
                    out.append(f"# HELP {name} {self._help[name][0]}\n# TYPE {name} histogram")
                    seen.add(name)
                acc = 0
                base = lbl[1:-1] if lbl else ""
                for b, c in zip(_BUCKETS, counts):
                    acc += c
                    sep = "," if base else ""
                    out.append(f'{name}_bucket{{{base}{sep}le="{b}"}} {acc}')
                sep = "," if base else ""
                out.append(f'{name}_bucket{{{base}{sep}le="+Inf"}} {n}')
                out.append(f"{name}_sum{lbl} {s}")
                out.append(f"{name}_count{lbl} {n}")
        return "\n".join(out) + "\n"


REGISTRY = Registry()

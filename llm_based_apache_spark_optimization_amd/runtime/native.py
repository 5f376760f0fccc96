"""Loader for the native host runtime (``_lsa_runtime``: scheduler, KV allocator, edit distance).

The extension is built in-tree by ``ops.build.build_runtime`` (g++, a few seconds).  A fresh checkout
builds it on first import; only if no C++ toolchain is present does it fall back to the equivalent
pure-Python classes below (identical semantics, used by nothing on the hot path).
"""
from __future__ import annotations

import collections
import importlib
import logging

log = logging.getLogger(__name__)


def _load():
    try:
        return importlib.import_module(__package__ + "._lsa_runtime")
    except ImportError:
        pass
    try:
        from ..ops.build import build_runtime

        build_runtime()
        return importlib.import_module(__package__ + "._lsa_runtime")
    except Exception as e:  # noqa: BLE001
        log.warning("native runtime unavailable (%s); using the Python fallback", e)
        return None


_mod = _load()
NATIVE = _mod is not None


class _PyBlockAllocator:
    def __init__(self, num_blocks: int, block_size: int = 64):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks (block 0 is scratch)")
        self.num_blocks, self.block_size = num_blocks, block_size
        self._free = list(range(num_blocks - 1, 0, -1))
        self._owned = set()

    def blocks_for(self, tokens):
        return (tokens + self.block_size - 1) // self.block_size

    def can_alloc(self, n):
        return len(self._free) >= n

    def alloc(self, n):
        if n < 0:
            raise ValueError("negative block count")
        if not self.can_alloc(n):
            raise RuntimeError("KV cache exhausted")
        if n == 0:
            return []
        out = self._free[-n:][::-1]
        del self._free[-n:]
        self._owned.update(out)
        return out

    def release(self, blocks):
        blocks = list(blocks)
        if any(b <= 0 or b >= self.num_blocks or b not in self._owned for b in blocks):
            raise ValueError("bad or already-free block id")
        if len(set(blocks)) != len(blocks):
            raise ValueError("block listed twice")
        for b in blocks:
            self._owned.discard(b)
            self._free.append(b)

    @property
    def num_free(self):
        return len(self._free)


class _PyScheduler:
    """Pure-Python twin of csrc/runtime/runtime_core.h Scheduler (lazy KV reservation + preemption)."""

    def __init__(self, num_blocks, block_size, max_slots, max_prefill_tokens, max_blocks_per_seq, reserve_tokens=64):
        self._alloc = _PyBlockAllocator(num_blocks, block_size)
        self._max_slots, self._budget, self._maxb = max_slots, max_prefill_tokens, max_blocks_per_seq
        self._reserve = reserve_tokens
        self._slots = [-1] * max_slots
        self._waiting = collections.deque()
        self._reqs = {}
        self._admits = 0

    def add(self, rid, prompt_len, max_new):
        if rid in self._reqs:
            raise ValueError("duplicate request id")
        if prompt_len < 1 or max_new < 1:
            raise ValueError("empty prompt or max_new < 1")
        need = self._alloc.blocks_for(prompt_len + max_new)
        if need > self._maxb:
            raise ValueError("request exceeds max model length")
        if need > self._alloc.num_blocks - 1:
            raise ValueError("request larger than the whole KV cache")
        self._reqs[rid] = {"p": prompt_len, "n": max_new, "slot": -1, "blocks": [], "seq": -1}
        self._waiting.append(rid)

    def _admit_blocks(self, r):
        gen = r["n"] if self._reserve < 0 else min(r["n"], self._reserve)
        return self._alloc.blocks_for(r["p"] + gen)

    def admit(self):
        out, budget = [], self._budget
        while self._waiting:
            r = self._reqs[self._waiting[0]]
            if out and r["p"] > budget:
                break
            need = self._admit_blocks(r)
            if not self._alloc.can_alloc(need):
                break
            try:
                slot = self._slots.index(-1)
            except ValueError:
                break
            rid = self._waiting.popleft()
            self._admits += 1
            r["blocks"], r["slot"], r["seq"] = self._alloc.alloc(need), slot, self._admits
            self._slots[slot] = rid
            budget -= r["p"]
            out.append(rid)
        return out

    def grow(self, rid, tokens):
        r = self._reqs[rid]
        if r["slot"] < 0:
            raise ValueError("grow: request is not running")
        want = min(self._alloc.blocks_for(min(tokens, r["p"] + r["n"])), self._maxb)
        add = want - len(r["blocks"])
        if add <= 0:
            return 0
        if not self._alloc.can_alloc(add):
            return -1
        r["blocks"] += self._alloc.alloc(add)
        return add

    def preempt(self, rid, prompt_len, max_new):
        r = self._reqs[rid]
        if r["slot"] < 0:
            raise ValueError("preempt: request is not running")
        if prompt_len < 1 or max_new < 1 or self._alloc.blocks_for(prompt_len + max_new) > self._maxb:
            raise ValueError("preempt: bad resumed lengths")
        self._slots[r["slot"]] = -1
        self._alloc.release(r["blocks"])
        r.update(slot=-1, blocks=[], seq=-1, p=prompt_len, n=max_new)
        self._waiting.appendleft(rid)

    def youngest_first(self):
        return sorted((s for s in self._slots if s >= 0), key=lambda rid: -self._reqs[rid]["seq"])

    def finish(self, rid):
        r = self._reqs.pop(rid, None)
        if r is None:
            return
        if r["slot"] >= 0:
            self._slots[r["slot"]] = -1
        if r["blocks"]:
            self._alloc.release(r["blocks"])
        if rid in self._waiting:
            self._waiting.remove(rid)

    def block_table(self, rid):
        return list(self._reqs[rid]["blocks"])

    def slot(self, rid):
        return self._reqs[rid]["slot"]

    def slot_owners(self):
        return list(self._slots)

    def running(self):
        return [s for s in self._slots if s >= 0]

    @property
    def num_waiting(self):
        return len(self._waiting)

    @property
    def num_running(self):
        return sum(1 for s in self._slots if s >= 0)

    @property
    def highest_slot(self):
        for i in range(self._max_slots - 1, -1, -1):
            if self._slots[i] >= 0:
                return i
        return -1

    @property
    def kv_usage(self):
        return 1.0 - self._alloc.num_free / (self._alloc.num_blocks - 1)

    @property
    def free_blocks(self):
        return self._alloc.num_free

    @property
    def reserve_tokens(self):
        return self._reserve


def _py_levenshtein(a: str, b: str) -> int:
    if len(a) < len(b):
        a, b = b, a
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i]
        for j, cb in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
        prev = cur
    return prev[-1]


if NATIVE:
    Scheduler = _mod.Scheduler
    BlockAllocator = _mod.BlockAllocator
    levenshtein = _mod.levenshtein
    levenshtein_batch = _mod.levenshtein_batch
else:  # pragma: no cover - only without a C++ toolchain
    Scheduler = _PyScheduler
    BlockAllocator = _PyBlockAllocator
    levenshtein = _py_levenshtein

    def levenshtein_batch(a, b):
        return [_py_levenshtein(x, y) for x, y in zip(a, b)]

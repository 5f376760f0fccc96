"""Build an LLMEngine for a named model (random-init or a checkpoint directory)."""
from __future__ import annotations

import time
from typing import Optional

import torch

from ..models import get_spec, tokenizer_for
from ..models.llama import init_random, load_safetensors_dir
from .engine import LLMEngine
from .runner import ModelRunner


def build_engine(model: str, device: Optional[str] = None, checkpoint: Optional[str] = None, dtype: str = "bf16",
                 max_slots: int = 32, max_model_len: int = 4096, seed: int = 0, tp=None,
                 use_graphs: bool = True, sync_every: int = 8, num_kv_blocks: Optional[int] = None,
                 max_prefill_tokens: int = 16384, kv_memory_fraction: float = 0.85,
                 warm_graphs: bool = False, prefill_chunk: Optional[int] = None,
                 kv_dtype: Optional[str] = None, max_new_cap: Optional[int] = None,
                 kv_reserve_tokens: int = 64) -> LLMEngine:
    """kv_dtype: paged KV cache dtype, "bf16" | "fp8" (None: LSA_KV_FP8, default bf16).
    max_new_cap: generated-token cap per request (None: the context window).
    kv_reserve_tokens: generated tokens whose KV is reserved at admission (the rest grows lazily; < 0 reserves
    prompt + max_new up front)."""
    if device is None:
        device = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu"
    t0 = time.perf_counter()
    tpr, tps = (tp.rank, tp.size) if tp is not None else (0, 1)
    if checkpoint:
        w = load_safetensors_dir(checkpoint, device, kind=dtype, name=model, tp_rank=tpr, tp_size=tps)
        tok = tokenizer_for(w.spec, checkpoint)
    else:
        spec = get_spec(model)
        w = init_random(spec, device, seed=seed, kind=dtype, tp_rank=tpr, tp_size=tps)
        tok = tokenizer_for(spec)
    runner = ModelRunner(w, max_slots=max_slots, max_model_len=max_model_len, tp=tp, use_graphs=use_graphs,
                         num_kv_blocks=num_kv_blocks, kv_memory_fraction=kv_memory_fraction, kv_dtype=kv_dtype,
                         max_new_cap=max_new_cap)
    eng = LLMEngine(runner, tok, sync_every=sync_every, max_prefill_tokens=max_prefill_tokens, name=model,
                    prefill_chunk=prefill_chunk or None, kv_reserve_tokens=kv_reserve_tokens)
    if torch.device(device).type == "cuda":
        if warm_graphs:
            runner.capture_all()
        torch.cuda.synchronize(device)
    eng.load_time_s = time.perf_counter() - t0
    return eng

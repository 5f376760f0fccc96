#!/usr/bin/env python3
"""Flagship benchmark: NL->SQL serving throughput + end-to-end latency on MI355X.

Metric (BASELINE.json): output tokens/sec + p50 end-to-end latency, duckdb-nsql-7B (default) or
Llama-3.2-3B (``--model llama3.2``).  One "step" = one complete serving round of ``--batch``
requests per replica: packed prefill of synthetic ``--prompt-len``-token prompts + ``--new-tokens``
greedy decode tokens (EOS ignored, so every request emits exactly that many tokens), i.e. the
request's end-to-end latency.  Random-init weights of the named architecture (no checkpoints can be
downloaded), bf16 (or ``--dtype fp8`` weights).

    python bench.py                      # 1 GPU, defaults
    torchrun --nproc-per-node 8 bench.py --gpus 8     # 8 DP replicas of one GPU each (dp8)
    torchrun --nproc-per-node 8 bench.py --gpus 8 --tp 2   # BASELINE config 4: 4 replicas x TP2 (tp2dp4)

Before the timed region one request of the first warm-up round is checked against the plain fp32
PyTorch forward over the same weights (``models.llama.reference_forward``, teacher-forced: every chosen
token must be within bf16 noise of the oracle's argmax); the result is reported as ``numerics``.

Prints ONE JSON line on rank 0.  ``value`` = whole-job output tokens/s (sum over replicas, timed by
the slowest rank); ``vs_baseline`` = value / 4.0 tok/s, the only throughput figure BASELINE.md
derives for the reference (its measured numbers are latencies: ``vs_baseline_p50_latency`` =
5.2381 s / our p50).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

REF_TOK_S = 4.0        # "<= 4 tok/s end-to-end for duckdb-nsql" (derived)
REF_P50_S = 5.2381     # duckdb-nsql p50 end-to-end latency, run B
REF_P50_S_LLAMA = 22.7463

MODEL_NAMES = {"duckdb-nsql": "duckdb-nsql-7B", "llama3.2": "Llama-3.2-3B-Instruct", "mistral": "Mistral-7B-v0.3"}


def fp8_label(r, B):
    """Which decode GEMMs of an fp8 model run W8A8 (fp8 activations) at batch B (engine/runner.py)."""
    xf = r.a8 and r.use_xfrag(B) and not (r.fused_norm and B <= r.fused_norm_max_batch)
    a8 = [name for name, on in (("qkv", xf and B > r.a8_min_batch), ("gate_up", xf and B > r.a8_mlp_min_batch)) if on]
    if not a8:
        return "fp8 (prefill W8A8 on fp8 MFMA, decode W8A16)"
    return f"fp8 (prefill W8A8 on fp8 MFMA; decode {' / '.join(a8)} W8A8 on fp8 MFMA, the rest W8A16)"


def check_numerics(eng, prompt, tokens, n=16, prefill_rows=0, decode_batch=0):
    """Teacher-forced check of the first ``n`` generated tokens against the fp32 reference forward:
    gap = (oracle max logit - oracle logit of our token) / oracle logit std, worst over the tokens.
    fp8 weights: the prompt rows get the W8A8 prefill's per-token activation rounding in the oracle when
    the packed prefill had > 64 rows (``prefill_rows``), as the engine's kernels do."""
    from llm_based_apache_spark_optimization_amd import ops
    from llm_based_apache_spark_optimization_amd.models.llama import reference_forward

    toks = list(tokens[:n])
    fp8 = eng.runner.w.layers[0].wqkv.kind == "fp8"
    aq = len(prompt) if (fp8 and prefill_rows > 64 and ops.FP8_W8A8) else 0
    r = eng.runner
    unfused_xf = bool(decode_batch and r.a8 and r.use_xfrag(decode_batch) and not (
        r.fused_norm and decode_batch <= r.fused_norm_max_batch))
    da8 = unfused_xf and decode_batch > r.a8_min_batch  # decode qkv W8A8
    da8m = unfused_xf and decode_batch > r.a8_mlp_min_batch  # decode gate_up W8A8
    lg = reference_forward(r.w, list(prompt) + toks[:-1], act_quant_rows=aq, decode_a8=da8,
                           decode_a8_mlp=da8m, kv_fp8=r.kv_fp8)[len(prompt) - 1:]
    chosen = lg.gather(1, torch.tensor(toks, device=lg.device).view(-1, 1)).squeeze(1)
    gap = ((lg.max(1).values - chosen) / lg.std(1)).max().item()
    agree = int((lg.argmax(1).cpu() == torch.tensor(toks)).sum())
    del lg
    if r.kv_fp8:
        # fp8 KV cache: every cached key / value row is rounded to e4m3 in the engine and in the oracle, from
        # values that differ at the bf16 level, so rows near a rounding boundary differ by a full e4m3 step; over
        # 32 layers on random-init weights (leading logits within a fraction of a std) that flips near-ties.
        # Per-layer parity at the strict criterion is pinned by tests/test_kv_fp8_gpu.py (2-layer prod shapes)
        ok, crit = gap < 1.0, "fp8 KV cache: gap < 1.0 std (quantisation-level; top-1 agreement reported)"
    elif aq or da8 or da8m:
        # W8A8 prefill: every prompt activation is rounded to e4m3 (3 mantissa bits); the oracle rounds the
        # same rows, but values near a rounding boundary land on different sides in the two computations, so
        # the prompt's K/V differ by quantisation-level noise that 32 layers accumulate.  On random-init
        # weights the leading logits sit within a fraction of a std of each other, so the criterion is the
        # quantisation-level one: every chosen token within 1 std of the oracle's best, half of them its argmax
        ok, crit = gap < 1.0 and agree >= len(toks) // 2, "W8A8: gap < 1.0 std, >= half top-1"
    else:
        ok, crit = gap < 0.15, "gap < 0.15 std"
    return {"tokens_checked": len(toks), "argmax_agree": agree, "max_gap_in_logit_std": round(gap, 4),
            "ok": ok, "criterion": crit}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="duckdb-nsql")
    ap.add_argument("--batch", type=int, default=32, help="requests per replica per step")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--new-tokens", type=int, default=128)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--kv-dtype", default=None, choices=["bf16", "fp8"],
                    help="paged KV cache dtype (default bf16; fp8 = e4m3 rows with per-row scales, ops.KV_FP8)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="run the same bench flow on CPU over gloo (tests of the multi-rank path; not a measurement)")
    args = ap.parse_args()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from llm_based_apache_spark_optimization_amd.engine import build_engine, SamplingParams
    from llm_based_apache_spark_optimization_amd.parallel import init_distributed, make_replica_groups

    cpu = args.cpu_rehearsal
    rank, world, local = init_distributed("gloo" if cpu else None)
    if cpu:
        device = torch.device("cpu")
    else:
        if not torch.cuda.is_available():
            print("bench.py needs a GPU", file=sys.stderr)
            return 2
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    if world != args.gpus and not cpu:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}; launch with torchrun "
              f"--nproc-per-node {args.gpus}", file=sys.stderr)
        return 2
    tp = max(1, args.tp)
    if world % tp:
        print(f"bench.py: WORLD_SIZE {world} not divisible by --tp {tp}", file=sys.stderr)
        return 2
    replica, tpg = make_replica_groups(world, tp, rank, device) if world > 1 else (0, None)
    dp = world // tp

    max_len = args.prompt_len + args.new_tokens + 64
    eng = build_engine(args.model, device=str(device), dtype=args.dtype, max_slots=args.batch,
                       max_model_len=max_len, seed=0, tp=tpg, use_graphs=not args.no_graphs,
                       max_prefill_tokens=max(16384, args.batch * args.prompt_len), kv_dtype=args.kv_dtype)
    V = eng.spec.vocab_size
    g = torch.Generator().manual_seed(1234 + replica)
    prompts = [[eng.spec.bos_id if eng.spec.bos_id < V else 1]
               + torch.randint(3, V, (args.prompt_len - 1,), generator=g).tolist() for _ in range(args.batch)]
    params = SamplingParams(max_tokens=args.new_tokens, temperature=0.0, ignore_eos=True)

    def one_step():
        res = eng.generate(prompts, params)
        assert all(r.eval_count == args.new_tokens for r in res), [r.eval_count for r in res]
        return res

    numerics = None
    for i in range(args.warmup):
        res = one_step()
        if i == 0 and tp == 1:
            numerics = check_numerics(eng, prompts[0], res[0].token_ids, prefill_rows=args.batch * args.prompt_len,
                                      decode_batch=args.batch)
    eng.stats.update(decode_s=0.0, decode_steps=0, prefill_s=0.0, decode_device_s=0.0)  # timed rounds only
    if world > 1:
        dist.barrier()
    sync()
    lat = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s = time.perf_counter()
        one_step()
        lat.append(time.perf_counter() - s)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], device=device)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    tokens = dp * args.batch * args.new_tokens * args.steps
    value = tokens / elapsed
    p50 = statistics.median(lat)
    ms_step = 1000.0 * elapsed / args.steps
    # GPU time per decode step from hipEvents around each decode run (excludes the prefill's kernels, which the
    # host-side decode_s also waits for: its first sync lands after the asynchronously launched prefill)
    decode_ms_tok = 1000.0 * eng.stats["decode_s"] / max(1, eng.stats["decode_steps"])
    decode_dev_ms = 1000.0 * eng.stats["decode_device_s"] / max(1, eng.stats["decode_steps"])
    if rank == 0:
        ref_p50 = REF_P50_S_LLAMA if args.model.startswith("llama") else REF_P50_S
        par = f"dp{dp}" if tp == 1 else f"tp{tp}dp{dp}"
        out = {
            "metric": "output_tokens_per_sec",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / REF_TOK_S, 2),
            "dtype": (args.dtype if args.dtype == "bf16" else fp8_label(eng.runner, args.batch))
            + ("; fp8 e4m3 KV cache" if eng.runner.kv_fp8 else ""),
            "data": "synthetic prompts, random-init weights" + (" (CPU rehearsal, not a measurement)" if cpu else ""),
            "config": {
                "model": MODEL_NAMES.get(args.model, args.model),
                "global_batch": dp * args.batch,
                "seq_len": args.prompt_len + args.new_tokens,
                "prompt_len": args.prompt_len,
                "new_tokens": args.new_tokens,
                "parallelism": par,
                "decode": "greedy",
            },
            "p50_e2e_latency_s": round(p50, 4),
            "vs_baseline_p50_latency": round(ref_p50 / p50, 2),
            "decode_ms_per_token_step": round(decode_ms_tok, 3),
            "decode_device_ms_per_step": round(decode_dev_ms, 3),
            "per_gpu_tokens_per_sec": round(value / world, 2),
            "numerics": numerics,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

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

Before the timed region the decode path is checked at the benchmark's batch (``eval/numerics.py``): the batch
is decoded greedily for 64 steps with each step's logits recorded, and two of its sequences are fed, with the
engine's own tokens, through the plain fp32 PyTorch forward over the same (for TP: the unsharded) weights
(``models.llama.reference_forward``, emulating fp8 quantisation where the engine quantises); mean KL, top-1 and
top-5 agreement over the 64 positions are reported as ``numerics``.

One-GPU runs then also time, untimed by the headline (after its region), BASELINE config 2 (the same model at
batch 1: ``p50_e2e_latency_s_b1``, ``decode_device_ms_per_step_b1``) and config 3 (Llama-3.2-3B /explain_error
with a 2k-token prompt, batch 1: ``explain_2k_p50_e2e_latency_s``, ``explain_2k_device_ms_per_step``), each with
its own teacher-forced numerics check (``--no-extras`` skips them).

Prints ONE JSON line on rank 0.  ``value`` = whole-job output tokens/s (sum over replicas, timed by
the slowest rank); ``vs_baseline`` = value / 4.0 tok/s, the only throughput figure BASELINE.md
derives for the reference (its measured numbers are latencies: ``vs_baseline_p50_latency`` =
5.2381 s / our p50).
"""
from __future__ import annotations

import argparse
import gc
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
    a8 = [name for name, on in zip(("qkv", "gate_up", "o", "down"), r.a8_plan(B)) if on]
    if r.w.layers[0].wqkv.kind == "mxfp4":
        if a8:
            return (f"mxfp4 weights (e2m1 + E8M0 per 32; decode {' / '.join(a8)} W4A8: e2m1 weights and e4m3 "
                    "activations straight into the block-scaled fp8 MFMA; prefill on the dequantised bf16 layer)")
        return ("mxfp4 weights (e2m1 + E8M0 per 32, decode W4A16: dequantised to bf16 in registers, bf16 MFMA; "
                "prefill on the dequantised bf16 layer), bf16 activations")
    if not a8:
        return "fp8 (prefill W8A8 on fp8 MFMA, decode W8A16)"
    return f"fp8 (prefill W8A8 on fp8 MFMA; decode {' / '.join(a8)} W8A8 on fp8 MFMA, the rest W8A16)"


def apply_overrides(eng, items) -> dict:
    """--set NAME=VALUE experiment overrides: ModelRunner attributes, or ops.NAME module constants."""
    import ast

    from llm_based_apache_spark_optimization_amd import ops

    out = {}
    for it in items:
        k, v = it.split("=", 1)
        try:
            val = ast.literal_eval(v)
        except (ValueError, SyntaxError):
            val = v
        if k.startswith("ops."):
            assert hasattr(ops, k[4:]), k
            setattr(ops, k[4:], val)
        else:
            assert hasattr(eng.runner, k), k
            setattr(eng.runner, k, val)
        out[k] = val
    return out


def numerics_check(eng, prompts, n_steps, rank0: bool, tp: int, model: str, dtype: str, device):
    """Teacher-forced check of the decode path at the benchmark's batch (eval/numerics.py): every rank runs the
    recording decode (TP ranks in lockstep), global rank 0 compares rows against the fp32 oracle over the
    UNSHARDED weights (TP engines hold one shard: the oracle regenerates the full seeded weights)."""
    from llm_based_apache_spark_optimization_amd.eval import numerics as nm

    toks, elog = nm.record_decode_logits(eng, prompts, n_steps)
    if not rank0:
        return None
    weights = None
    if tp > 1:
        from llm_based_apache_spark_optimization_amd.models import get_spec
        from llm_based_apache_spark_optimization_amd.models.llama import init_random

        weights = init_random(get_spec(model), device, seed=0, kind=dtype)
    res = nm.check_recorded(eng, prompts, toks, elog, n_steps, check_rows=(0, len(prompts) - 1), weights=weights)
    del weights, elog
    return res


def _timed_rounds(eng, prompts, params, n: int):
    """n untimed-by-the-headline rounds: (p50 e2e latency s, GPU ms per decode step)."""
    import statistics as st

    eng.generate(prompts, params)  # warm (graphs of this bucket captured)
    eng.stats.update(decode_s=0.0, decode_steps=0, prefill_s=0.0, decode_device_s=0.0)
    lat = []
    for _ in range(n):
        t = time.perf_counter()
        res = eng.generate(prompts, params)
        lat.append(time.perf_counter() - t)
        assert all(r.eval_count == params.max_tokens for r in res)
    return st.median(lat), 1000.0 * eng.stats["decode_device_s"] / max(1, eng.stats["decode_steps"])


def batch1_round(eng, prompt, args) -> dict:
    """BASELINE config 2 on the same engine: one request, ``--new-tokens`` greedy tokens (the reference's own
    per-request shape, Model_Evaluation_&_Comparision.py:113-119)."""
    from llm_based_apache_spark_optimization_amd.engine import SamplingParams

    num = numerics_check(eng, [prompt], min(64, args.new_tokens - 1), True, 1, args.model, args.dtype, None)
    p50, dev = _timed_rounds(eng, [prompt], SamplingParams(max_tokens=args.new_tokens, temperature=0.0,
                                                           ignore_eos=True), 5)
    return {"p50_e2e_latency_s_b1": round(p50, 4), "decode_device_ms_per_step_b1": round(dev, 3),
            "vs_baseline_p50_latency_b1": round(REF_P50_S / p50, 2), "numerics_b1": num}


def explain_round(device, prompt_len: int = 2048, new_tokens: int = 128) -> dict:
    """BASELINE config 3: Llama-3.2-3B-Instruct /explain_error, a ``prompt_len``-token synthetic Spark stack
    trace, batch 1, bf16 (Flask/app.py:153-164)."""
    from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine

    eng = build_engine("llama3.2", device=str(device), dtype="bf16", max_slots=2,
                       max_model_len=prompt_len + new_tokens + 64, seed=0)
    g = torch.Generator().manual_seed(4321)
    prompt = [eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (prompt_len - 1,), generator=g).tolist()
    num = numerics_check(eng, [prompt], 64, True, 1, "llama3.2", "bf16", None)
    p50, dev = _timed_rounds(eng, [prompt], SamplingParams(max_tokens=new_tokens, temperature=0.0, ignore_eos=True), 3)
    # time to first token: a one-token request (2k-token prefill + first-token commit + the host read-back)
    ttft = []
    for _ in range(3):
        t = time.perf_counter()
        eng.generate([prompt], SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
        ttft.append(time.perf_counter() - t)
    out = {"explain_2k_p50_e2e_latency_s": round(p50, 4), "explain_2k_device_ms_per_step": round(dev, 3),
           "explain_2k_ttft_s": round(sorted(ttft)[1], 4),
           "vs_baseline_p50_latency_explain": round(REF_P50_S_LLAMA / p50, 2), "numerics_explain_2k": num,
           "explain_2k_config": {"model": MODEL_NAMES["llama3.2"], "prompt_len": prompt_len, "new_tokens": new_tokens,
                                 "batch": 1, "dtype": "bf16"}}
    del eng
    gc.collect()
    torch.cuda.empty_cache()
    return out


def comm_record(tpg, world: int, tp: int, device) -> dict:
    """Self-verifying record of how the ranks communicated (collective over the world): every rank's device, and
    per TP group the backend, ranks per group, whether the one-shot IPC all-reduce ran (else why not) and the
    issued collectives per path -- so a scaling run shows N ranks on N distinct GPUs and which TP path it timed."""
    mine = {"rank": dist.get_rank(), "device": str(device),
            "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES"),
            "tp": tpg.describe() if tpg is not None else None}
    recs: list = [None] * world
    dist.all_gather_object(recs, mine)
    devs = [r["device"] for r in recs]
    out = {"world": world, "tp": tp, "backend": dist.get_backend(), "device_per_rank": devs,
           "distinct_devices": len(set(devs))}
    if tp > 1:
        groups = [r["tp"] for r in recs]
        calls: dict = {}
        for g in groups:
            for k, v in g["calls"].items():
                calls[k] = calls.get(k, 0) + v
        out.update({"tp_backend": groups[0]["backend"], "group_ranks": sorted({g["group_ranks"] for g in groups}),
                    "ipc_allreduce": all(g["ipc_allreduce"] for g in groups),
                    "ipc_bf16_payload": groups[0]["ipc_bf16_payload"],
                    "ipc_fallback": sorted({g["ipc_fallback"] for g in groups if g["ipc_fallback"]}) or None,
                    "calls_all_ranks": dict(sorted(calls.items()))})
    return out


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
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "mxfp4"],
                    help="weights: bf16 | fp8 (e4m3, per-channel scales) | mxfp4 (OCP MX e2m1 + E8M0 block scales, the "
                         "4-bit weight class of the reference's Ollama tags; W4A16 decode)")
    ap.add_argument("--kv-dtype", default=None, choices=["bf16", "fp8"],
                    help="paged KV cache dtype (default bf16; fp8 = e4m3 rows with per-row scales, ops.KV_FP8)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="run the same bench flow on CPU over gloo (tests of the multi-rank path; not a measurement)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the untimed BASELINE config 2 (batch 1) / config 3 (3B 2k explain) rounds after the "
                         "timed region (they run on one-GPU-per-replica GPU benches by default)")
    ap.add_argument("--set", action="append", default=[], metavar="NAME=VALUE",
                    help="experiment override (A/B runs; reported as 'overrides'): a ModelRunner attribute, or "
                         "ops.NAME for a module constant of ops, e.g. --set fused_norm_max_batch=32")
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
    overrides = apply_overrides(eng, args.set)
    V = eng.spec.vocab_size
    g = torch.Generator().manual_seed(1234 + replica)
    prompts = [[eng.spec.bos_id if eng.spec.bos_id < V else 1]
               + torch.randint(3, V, (args.prompt_len - 1,), generator=g).tolist() for _ in range(args.batch)]
    params = SamplingParams(max_tokens=args.new_tokens, temperature=0.0, ignore_eos=True)

    def one_step():
        res = eng.generate(prompts, params)
        assert all(r.eval_count == args.new_tokens for r in res), [r.eval_count for r in res]
        return res

    # numerics before the warm-up: a teacher-forced decode of the same batch, >= 64 steps when the run has them
    numerics = numerics_check(eng, prompts, min(64, args.new_tokens - 1), rank == 0, tp, args.model, args.dtype, device)
    for i in range(args.warmup):
        one_step()
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
    tp_comm = comm_record(tpg, world, tp, device) if world > 1 else None
    decode_ms_tok = 1000.0 * eng.stats["decode_s"] / max(1, eng.stats["decode_steps"])
    decode_dev_ms = 1000.0 * eng.stats["decode_device_s"] / max(1, eng.stats["decode_steps"])
    extras = {}
    if world == 1 and not cpu and not args.no_extras:
        extras.update(batch1_round(eng, prompts[0], args))
        dtype_label = (args.dtype if args.dtype == "bf16" else fp8_label(eng.runner, args.batch)) \
            + ("; fp8 e4m3 KV cache" if eng.runner.kv_fp8 else "")
        del eng
        gc.collect()
        torch.cuda.empty_cache()
        extras.update(explain_round(device))
        eng = None
    else:
        dtype_label = (args.dtype if args.dtype == "bf16" else fp8_label(eng.runner, args.batch)) \
            + ("; fp8 e4m3 KV cache" if eng.runner.kv_fp8 else "")
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
            "dtype": dtype_label,
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
            **({"tp_comm": tp_comm} if tp_comm is not None else {}),
            **({"overrides": overrides} if overrides else {}),
            **extras,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

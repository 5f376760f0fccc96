"""Prefill A/B on MI355X: time-to-first-token of one request (prefill + first-token commit + read-back) with the
vendor residual GEMM (ops.PREFILL_BLAS_RES) and the small-M SiLU vendor route (ops.PREFILL_BLAS_SILU_MAX_M) on / off:
  3B 2k explain prompt (BASELINE config 3), 7B 300-token NL->SQL prompt, 7B 32 x 128 (the headline round's prefill).
Also a teacher-forced numerics check of the 3B with each setting.
    python scripts/bench_prefill_ab.py > gpurun_out/prefill_ab.jsonl
"""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

SP = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)


def ttft(eng, prompts, n=7):
    eng.generate(prompts, SP)
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.generate(prompts, SP)
        ts.append(time.perf_counter() - t)
    return round(statistics.median(ts) * 1e3, 3)


def prompts(eng, n, L, seed):
    g = torch.Generator().manual_seed(seed)
    return [[eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (L - 1,), generator=g).tolist() for _ in range(n)]


def main():
    SETTINGS = {"res": (True, 0, False), "res+silu": (True, 1024, False), "res+silu16": (True, 1024, True),
                "res+silu16_all": (True, 1 << 30, True)}
    for model, n, L in (("llama3.2", 1, 2048), ("duckdb-nsql", 1, 300), ("duckdb-nsql", 32, 128)):
        eng = build_engine(model, device="cuda:0", dtype="bf16", max_slots=max(2, n), max_model_len=L + 64, seed=0)
        ps = prompts(eng, n, L, 99)
        for name, (res, silu, s16) in SETTINGS.items():
            ops.PREFILL_BLAS_RES = res
            ops.PREFILL_BLAS_SILU_MAX_M = silu
            ops.PREFILL_BLAS_SILU_BF16 = s16
            out = {"model": model, "prompts": n, "len": L, "setting": name, "ttft_ms": ttft(eng, ps)}
            if n == 1 and L == 2048:
                from llm_based_apache_spark_optimization_amd.eval import numerics
                num = numerics.teacher_forced_check(eng, ps, n_steps=8)
                out.update(ok=num["ok"], hidden_rel_err=num.get("hidden_rel_err"), probe_kl=num.get("probe_kl"))
            print(json.dumps(out), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

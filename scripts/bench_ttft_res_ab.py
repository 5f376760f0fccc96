"""TTFT with the prefill o / down vendor GEMMs accumulating into the f32 residual (ops.PREFILL_BLAS_RES) on / off,
interleaved reps on one box: 3B 2k explain prompt and the 7B 32 x 128 headline round's prefill.
    python scripts/bench_ttft_res_ab.py > gpurun_out/ttft_res_ab.jsonl
"""
import json
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts")
from bench_prefill_ab import prompts, ttft  # noqa: E402

from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import build_engine  # noqa: E402

for model, n, L in (("llama3.2", 1, 2048), ("duckdb-nsql", 32, 128)):
    eng = build_engine(model, device="cuda:0", dtype="bf16", max_slots=max(2, n), max_model_len=L + 64, seed=0)
    ps = prompts(eng, n, L, 99)
    for rep in range(3):
        for res in (False, True):
            ops.PREFILL_BLAS_RES = res
            print(json.dumps({"model": model, "prompts": n, "len": L, "rep": rep, "blas_res": res,
                              "ttft_ms": ttft(eng, ps)}), flush=True)
    ops.PREFILL_BLAS_RES = True
    del eng
    torch.cuda.empty_cache()

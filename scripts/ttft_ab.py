"""Time to first token of the BASELINE config-3 request (Llama-3.2-3B-Instruct, 2048-token prompt, batch 1) under
prefill-path switches, interleaved in one process: ops.ROPE_FUSED (RoPE + KV append in the qkv GEMM epilogue) and
ops.RES_FUSED (residual add in the o / down GEMM epilogues).  Prints one JSON line per arm (median of rounds)."""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "llama3.2"
plen = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
eng = build_engine(model, device="cuda:0", dtype="bf16", max_slots=2, max_model_len=plen + 128, seed=0)
g = torch.Generator().manual_seed(4321)
prompt = [eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
sp = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
arms = {"rope1_res1": (True, True), "rope0_res1": (False, True), "rope1_res0": (True, False),
        "rope0_res0": (False, False)}
times = {a: [] for a in arms}
for rnd in range(6):
    for a, (rope, res) in arms.items():
        ops.ROPE_FUSED, ops.RES_FUSED, ops.ROPE_FUSED_MIN_M = rope, res, 0
        t = time.perf_counter()
        eng.generate([prompt], sp)
        dt = time.perf_counter() - t
        if rnd > 0:
            times[a].append(dt)
for a in arms:
    print(json.dumps({"model": model, "prompt_len": plen, "arm": a, "ttft_ms": round(1000 * statistics.median(times[a]), 2),
                      "min_ms": round(1000 * min(times[a]), 2)}), flush=True)

"""3B time to first token on a long prompt with the RoPE-epilogue qkv GEMM on its measured "rope" tile configuration
(ops.rope_config) vs the bf16 entry's tile widened to 256 columns (the route before the rope entries), arms interleaved.
    python scripts/ttft_rope_cfg_ab.py [model] [prompt_len]
"""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "llama3.2"
plen = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
eng = build_engine(model, device="cuda:0", dtype="bf16", max_slots=2, max_model_len=plen + 128, seed=0)
g = torch.Generator().manual_seed(4321)
prompt = [eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
sp = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
table = ops.rope_config
arms = {"rope_entry": table, "bf16_entry": lambda M, N, K: ops.sk_config(M, N, K, "bf16")}
times = {a: [] for a in arms}
first = {}
for rnd in range(7):
    for a, fn in arms.items():
        ops.rope_config = fn
        t = time.perf_counter()
        out = eng.generate([prompt], sp)
        dt = time.perf_counter() - t
        first[a] = out[0].token_ids[0]
        if rnd > 1:
            times[a].append(dt)
for a in arms:
    print(json.dumps({"model": model, "prompt_len": plen, "arm": a, "ttft_ms": round(1000 * statistics.median(times[a]), 2),
                      "min_ms": round(1000 * min(times[a]), 2), "first_token": first[a]}), flush=True)

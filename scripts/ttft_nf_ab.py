"""Time to first token with the norm-free attention input on / off (engine.runner.PREFILL_NORM_FREE: the down
stream-K epilogue writes bf16(h) + the Q24 row sums of h^2 and the qkv GEMM scales its output rows, vs the
attention-side add_rmsnorm launch of every layer), interleaved in one process on the BASELINE config-3 request (Llama-3.2-3B-Instruct,
2048-token prompt, batch 1) by default.  Prints one JSON line per arm (median of rounds) and whether the arms
picked the same first token.
    python scripts/ttft_nf_ab.py [model] [prompt_len] [arm]    (arm nf1 | nf0: that arm alone, e.g. under rocprofv3)
"""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import runner  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "llama3.2"
plen = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
eng = build_engine(model, device="cuda:0", dtype="bf16", max_slots=2, max_model_len=plen + 128, seed=0)
g = torch.Generator().manual_seed(4321)
prompt = [eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
sp = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
arms = {"nf1": True, "nf0": False}
if len(sys.argv) > 3:
    arms = {sys.argv[3]: arms[sys.argv[3]]}
times = {a: [] for a in arms}
first = {}
for rnd in range(8):
    for a, on in arms.items():
        runner.PREFILL_NORM_FREE = on
        t = time.perf_counter()
        out = eng.generate([prompt], sp)
        dt = time.perf_counter() - t
        first[a] = out[0].token_ids[0] if hasattr(out[0], "token_ids") else str(out[0])
        if rnd > 1:
            times[a].append(dt)
for a in arms:
    print(json.dumps({"model": model, "prompt_len": plen, "arm": a, "ttft_ms": round(1000 * statistics.median(times[a]), 2),
                      "min_ms": round(1000 * min(times[a]), 2), "first_token": first[a]}), flush=True)

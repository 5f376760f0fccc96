"""A/B of the batch-1 decode step, residual-reduce (ModelRunner._decode_step_rr) vs the step it replaces, in one
process, arms interleaved (cdna_hip_programming.md §5.4 rule 24).  One JSON line per (arm, round), then a summary.

    python scripts/ab_decode_b1.py llama3.2 2048     # BASELINE config 3 (3B /explain_error, 2k prompt)
    python scripts/ab_decode_b1.py duckdb-nsql 128   # BASELINE config 2 (7B NL->SQL, batch 1)
    python scripts/ab_decode_b1.py duckdb-nsql 128 3 "" mxfp4   # the same with MXFP4 weights (W4A8 RR step)
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import _timed_rounds, numerics_check  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "llama3.2"
plen = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
only = (sys.argv[4] or None) if len(sys.argv) > 4 else None  # one arm (profiling runs)
dtype = sys.argv[5] if len(sys.argv) > 5 else "bf16"  # bf16 | fp8 | mxfp4 weights
new = 128
eng = build_engine(model, device="cuda:0", dtype=dtype, max_slots=2 if plen > 1024 else 32,
                   max_model_len=plen + new + 64, seed=0)
r = eng.runner
g = torch.Generator().manual_seed(4321)
prompt = [eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
sp = SamplingParams(max_tokens=new, temperature=0.0, ignore_eos=True)
arms = {k: v for k, v in {"rr": True, "norm_launch": False}.items() if only in (None, k)}
res = {k: [] for k in arms}
for k, on in arms.items():
    r.rr_decode = on
    r.graphs.clear()
    num = numerics_check(eng, [prompt], 64, True, 1, model, dtype, None)
    print(json.dumps({"arm": k, "numerics": num, "launches_b1": r.count_step_kernels(1)}), flush=True)
for i in range(rounds):
    for k, on in arms.items():
        r.rr_decode = on
        r.graphs.clear()
        p50, dev = _timed_rounds(eng, [prompt], sp, 3)
        res[k].append(dev)
        print(json.dumps({"arm": k, "round": i, "decode_device_ms_per_step": round(dev, 4), "p50_s": round(p50, 4)}),
              flush=True)
print(json.dumps({"model": model, "dtype": dtype, "prompt_len": plen, **{k: round(statistics.median(v), 4) for k, v in res.items()}}))

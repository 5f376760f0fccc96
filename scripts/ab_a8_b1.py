"""A/B of the batch-1 decode step of a quantised model: the default bucket plan (fp8: W8A16 GEMMs with norm launches)
vs every projection W8A8 / W4A8 at batch 1, which also enables the W8A8 residual-reduce step (ModelRunner.rr_a8:
qkv / gate_up quantise their own residual-reduced input, no norm launch).  Arms interleaved in one process
(cdna_hip_programming.md §5.4 rule 24); one JSON line per (arm, round), then a summary.

    python scripts/ab_a8_b1.py duckdb-nsql 128 fp8
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import _timed_rounds, numerics_check  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "duckdb-nsql"
plen = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dtype = sys.argv[3] if len(sys.argv) > 3 else "fp8"
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
new = 128
eng = build_engine(model, device="cuda:0", dtype=dtype, max_slots=2 if plen > 1024 else 32,
                   max_model_len=plen + new + 64, seed=0)
r = eng.runner
g = torch.Generator().manual_seed(4321)
prompt = [eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
sp = SamplingParams(max_tokens=new, temperature=0.0, ignore_eos=True)
base = (r.a8_min_batch, r.a8_mlp_min_batch, r.a8_od_max_batch)
arms = {"default": base, "a8_all_b1": (0, 0, max(1, base[2]))}
res = {k: [] for k in arms}
for k, bk in arms.items():
    r.set_a8_buckets(*bk)
    num = numerics_check(eng, [prompt], 64, True, 1, model, dtype, None)
    print(json.dumps({"arm": k, "buckets": bk, "a8_plan_b1": r.a8_plan(1), "rr_decode": r.rr_decode, "rr_a8": r.rr_a8,
                      "numerics": num, "launches_b1": r.count_step_kernels(1)}), flush=True)
for i in range(rounds):
    for k, bk in arms.items():
        r.set_a8_buckets(*bk)
        p50, dev = _timed_rounds(eng, [prompt], sp, 3)
        res[k].append(dev)
        print(json.dumps({"arm": k, "round": i, "decode_device_ms_per_step": round(dev, 4), "p50_s": round(p50, 4)}),
              flush=True)
r.set_a8_buckets(*base)
print(json.dumps({"model": model, "dtype": dtype, "prompt_len": plen,
                  **{k: round(statistics.median(v), 4) for k, v in res.items()}}))

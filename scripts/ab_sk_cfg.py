"""In-engine A/B of stream-K prefill GEMM table entries (ops/gemm_sk_tuning.json "NxK:epi:mB" -> cfg): time to first
token of one request (prefill + first-token commit + host read-back) with the table vs with each override set, arms
interleaved in one process (cdna_hip_programming.md §5.4 rule 24), median of the rounds.  The table was built from
standalone cold-cache sweeps; in the engine each GEMM runs after the previous layer's kernels.
Usage: ab_sk_cfg.py <model> <prompt_len> <requests> '<json list of {key: cfg} | {"ops:NAME": value}>' [rounds]"""
import copy
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

model, plen, nreq, ovs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), json.loads(sys.argv[4])
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 7
eng = build_engine(model, device="cuda:0", dtype="bf16", max_slots=max(2, nreq), max_model_len=plen + 128, seed=0,
                   max_prefill_tokens=max(16384, plen * nreq))
g = torch.Generator().manual_seed(4321)
prompts = [[eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
           for _ in range(nreq)]
sp = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
ops.sk_config(plen * nreq, 4096, 4096, "bf16")  # loads the table
base = copy.deepcopy(ops._sk_tuning)
arms = {"table": {}, **{f"ov{i}": o for i, o in enumerate(ovs)}}
times = {k: [] for k in arms}
ops0 = {}
for rnd in range(rounds + 1):
    for k, o in arms.items():
        # "ops:NAME" keys set an ops module attribute for the arm (e.g. ops:ROPE_FUSED_MIN_M)
        for name, v in ops0.items():
            setattr(ops, name, v)
        for key, v in o.items():
            if key.startswith("ops:"):
                ops0.setdefault(key[4:], getattr(ops, key[4:]))
                setattr(ops, key[4:], v)
        ops._sk_tuning = {**base, **{key: {"cfg": c} for key, c in o.items() if not key.startswith("ops:")}}
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.generate(prompts, sp)
        dt = time.perf_counter() - t
        if rnd > 0:
            times[k].append(dt)
ops._sk_tuning = base
for name, v in ops0.items():
    setattr(ops, name, v)
print(json.dumps({"model": model, "prompt_len": plen, "requests": nreq, "arms": {k: arms[k] for k in arms},
                  "ttft_ms": {k: round(1000 * statistics.median(v), 3) for k, v in times.items()},
                  "min_ms": {k: round(1000 * min(v), 3) for k, v in times.items()}}), flush=True)

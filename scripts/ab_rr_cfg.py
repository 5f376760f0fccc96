"""In-engine A/B of batch-1 decode GEMM tuning entries (first written for the residual-reduce (ops.rr_config "NxK:epi:b1:rr[:kind]" keys, from
scripts/sweep_rr_b1.py)): the decode step with the entries given as ops.TUNING_OVERRIDES vs without, arms interleaved
in one process, numerics of both.  A qkv entry also changes how many split-K slabs the attention prologue sums.
Usage: ab_rr_cfg.py <model> <prompt_len> <dtype> '<json overrides | json list of overrides>' [rounds]
(any decode tuning key may be overridden, e.g. the plain W4A8 down entry "4096x11008:f32:b1:fp4a")."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import _timed_rounds, numerics_check  # noqa: E402
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

model, plen, dtype, ov = sys.argv[1], int(sys.argv[2]), sys.argv[3], json.loads(sys.argv[4])
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 3
new = 128
eng = build_engine(model, device="cuda:0", dtype=dtype, max_slots=2 if plen > 1024 else 32,
                   max_model_len=plen + new + 64, seed=0)
r = eng.runner
print(json.dumps({"rr_decode": r.rr_decode, "rr_a8": r.rr_a8}), flush=True)  # fp8 b1: the norm-free W8A16 step
g = torch.Generator().manual_seed(4321)
batch = int(os.environ.get("AB_BATCH", "1"))  # decode batch (the bench's b32: AB_BATCH=32)
prompts = [[eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
           for _ in range(batch)]
sp = SamplingParams(max_tokens=new, temperature=0.0, ignore_eos=True)
arms = {"table": {}, **({f"ov{i}": o for i, o in enumerate(ov)} if isinstance(ov, list) else {"override": ov})}
res = {k: [] for k in arms}


attr0 = {}


def use(o):  # "plan:B:Hkv" keys override the split-KV decode plan (chunk_blocks, nsplit, unsplit_max); "attr:name"
    # keys set a ModelRunner attribute for the arm (e.g. attr:fused_norm_max_batch)
    for k, v in attr0.items():
        setattr(r, k, v)
    for k, v in o.items():
        if k.startswith("attr:"):
            attr0.setdefault(k[5:], getattr(r, k[5:]))
            setattr(r, k[5:], tuple(v) if isinstance(v, list) else v)
    ops.TUNING_OVERRIDES.clear()
    ops.TUNING_OVERRIDES.update({k: v for k, v in o.items() if not k.startswith(("plan:", "attr:"))})
    ops.DECODE_PLAN_OVERRIDES.clear()
    ops.DECODE_PLAN_OVERRIDES.update({tuple(int(x) for x in k.split(":")[1:]): tuple(v) for k, v in o.items()
                                      if k.startswith("plan:")})
    r.graphs.clear()


for k, o in arms.items():
    use(o)
    num = numerics_check(eng, prompts, 64, True, 1, model, dtype, None)
    print(json.dumps({"arm": k, "overrides": o, "numerics": num}), flush=True)
for i in range(rounds):
    for k, o in arms.items():
        use(o)
        p50, dev = _timed_rounds(eng, prompts, sp, 3)
        res[k].append(dev)
        print(json.dumps({"arm": k, "round": i, "decode_device_ms_per_step": round(dev, 4)}), flush=True)
use({})
print(json.dumps({"model": model, "dtype": dtype, "prompt_len": plen, "batch": batch, **{k: round(statistics.median(v), 4)
                                                                           for k, v in res.items()}}))

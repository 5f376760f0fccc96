"""Time to first token under a kernel knob, arms interleaved in one process (cdna_hip_programming.md §5.4 rule 24): a
one-token request (prefill + first-token commit + host read-back) for each case, median (and min) of the rounds.
Knob 'one_phase': the stream-K GEMM's one-phase K-loop schedule for the 128-row tiles (ext.gemm_sk_one_phase);
'prefill_xf': the fragment-major prefill activations (ops.PREFILL_XF); 'rope_fused_all': the RoPE / cache-append
qkv epilogue at every prefill size (1) vs from 4096 rows (0, the default); 'gateup300_256': the 7B gate_up table
entry at 300 rows, 256 x 256 whole tiles (1) vs 128 x 256 stream-K (0);
'none': one arm, the loaded build (cross-build A/Bs: run it under LSA_HIP_SO=variants/<name>.so in turns).
Usage: ttft_knob_ab.py [knob] [rounds] [case,...]"""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine  # noqa: E402

knob = sys.argv[1] if len(sys.argv) > 1 else "one_phase"


def _table_cfg(key, cfg):  # one stream-K tuning-table entry (ops.sk_config) overridden in place
    ops.sk_config(128, 128, 128, "bf16")  # loads the table
    ops._sk_tuning[key] = dict(ops._sk_tuning.get(key, {}), cfg=cfg)


rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
KNOBS = {"one_phase": lambda v: ops.ext().gemm_sk_one_phase(v), "none": lambda v: None,
         "prefill_xf": lambda v: setattr(ops, "PREFILL_XF", bool(v)),
         "rope_fused_all": lambda v: setattr(ops, "ROPE_FUSED_MIN_M", 65 if v else 4096),
         "gateup300_256": lambda v: _table_cfg("22016x4096:silu:m300", 24 if v else 19)}
setk = KNOBS[knob]
# (model, prompt tokens, requests in the batch): config 3 (3B explain, 2k prompt), config 2 (7B NL->SQL prompt),
# the headline bench's batch-32 prefill (32 x 128 tokens)
CASES = [("llama3.2", 2048, 1), ("duckdb-nsql", 300, 1), ("duckdb-nsql", 128, 32)]
if len(sys.argv) > 3:  # a subset, e.g. "0,1" (a cross-build A/B whose older build lacks a binding the last case uses)
    CASES = [CASES[int(i)] for i in sys.argv[3].split(",")]
sp = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
for model, plen, nreq in CASES:
    eng = build_engine(model, device="cuda:0", dtype="bf16", max_slots=max(2, nreq), max_model_len=plen + 128, seed=0,
                       max_prefill_tokens=max(16384, plen * nreq))
    g = torch.Generator().manual_seed(4321)
    prompts = [[eng.spec.bos_id] + torch.randint(3, eng.spec.vocab_size, (plen - 1,), generator=g).tolist()
               for _ in range(nreq)]
    times = {0: [], 1: []}
    for rnd in range(rounds + 1):
        for v in (0, 1):
            setk(v)
            torch.cuda.synchronize()
            t = time.perf_counter()
            eng.generate(prompts, sp)
            dt = time.perf_counter() - t
            if rnd > 0:
                times[v].append(dt)
    setk(1)
    print(json.dumps({"knob": knob, "model": model, "prompt_len": plen, "requests": nreq,
                      **{f"ttft_ms_{v}": round(1000 * statistics.median(times[v]), 2) for v in (0, 1)},
                      **{f"min_ms_{v}": round(1000 * min(times[v]), 2) for v in (0, 1)}}), flush=True)
    del eng
    torch.cuda.empty_cache()

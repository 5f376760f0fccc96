"""Build ops/gemm_sk_tuning.json from a bench_prefill_gemm.py --grid sweep (jsonl): for every (N, K, epilogue, M)
the fastest tile configuration of the stream-K prefill kernel (ops.SK_CFGS index, + 8 = whole tiles only) and, when the
sweep compared epilogue modes (arm suffix _e0 / _e1), the faster mode (stored as cfg + 16 + 32 * mode).
Usage: make_sk_tuning.py gpurun_out/bench_prefill_gemm.jsonl [more.jsonl ...]"""
import json
import os
import sys

CFG = {"256x256": 0, "256x192": 1, "256x128": 2, "128x256": 3, "128x192": 4, "128x128": 5, "128x192w4": 6,
       "128x128w4": 7}
out_path = os.path.join(os.path.dirname(__file__), "..", "llm_based_apache_spark_optimization_amd", "ops",
                        "gemm_sk_tuning.json")
tab = {}
try:
    with open(out_path) as f:
        tab = json.load(f)
except (OSError, ValueError):
    pass
for path in sys.argv[1:]:
    for line in open(path):
        r = json.loads(line)
        best, best_us = None, 1e30
        for k, v in r.items():
            if not (k.startswith("sk_") and isinstance(v, dict)) or "auto" in k or "table" in k:
                continue
            parts = k.split("_")
            tag = parts[1]
            dp = tag.endswith("dp")
            cfg = CFG[tag[:-2] if dp else tag] + (8 if dp else 0)
            if parts[-1] in ("e0", "e1"):
                cfg += 16 + 32 * int(parts[-1][1])
            if v["us"] < best_us:
                best, best_us = cfg, v["us"]
        if best is not None:
            epi = "res" if r["epi"] in ("res", "f32") else r["epi"]
            tab[f"{r['N']}x{r['K']}:{epi}:m{r['M']}"] = {"cfg": best, "us": best_us}
with open(out_path, "w") as f:
    json.dump(dict(sorted(tab.items())), f, indent=1)
print(f"{len(tab)} entries -> {out_path}")

"""Fold the "tune" entries of sweep JSON lines (scripts/bench_res_epi.py, ...) into ops/gemm_tuning.json.

    python scripts/merge_tuning.py gpurun_out/x/res_epi_bf16.jsonl [...]
"""
import json
import sys

PATH = "llm_based_apache_spark_optimization_amd/ops/gemm_tuning.json"
tab = json.load(open(PATH))
n = 0
for fn in sys.argv[1:]:
    for line in open(fn):
        line = line.strip()
        if not line.startswith("{"):
            continue
        for k, v in json.loads(line).get("tune", {}).items():
            tab[k] = v
            n += 1
json.dump(dict(sorted(tab.items())), open(PATH, "w"), indent=1, sort_keys=True)
open(PATH, "a").write("\n")
print(f"merged {n} entries into {PATH}")

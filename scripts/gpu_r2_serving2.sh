#!/bin/bash
# co-serving (BASELINE config 5) at HEAD: fixed-QPS phases, then the streaming TTFT run
export TMPDIR=/tmp
O=gpurun_out/serve3; mkdir -p $O
timeout -k 10 600 python -u -m llm_based_apache_spark_optimization_amd.bench_serving --qps 4,8,16,24,32 --duration 20 > $O/coserve.json 2> $O/coserve.err || { tail -n 30 $O/coserve.err; exit 1; }
timeout -k 10 600 python -u -m llm_based_apache_spark_optimization_amd.bench_serving --qps 4,8,16,24 --duration 20 --stream > $O/stream.json 2> $O/stream.err || { tail -n 30 $O/stream.err; exit 2; }
python3 - <<'PY'
import json
for f in ("gpurun_out/serve3/coserve.json", "gpurun_out/serve3/stream.json"):
    d = json.load(open(f))
    for ph in d["phases"]:
        n, e = ph["nl2sql"], ph["explain_error"]
        print(f, ph["qps_target"], ph["achieved_qps"], round(ph["output_tokens_per_sec"]), n["p50_s"], n["p99_s"], e["p50_s"], e["p99_s"],
              {k: v for k, v in ph.items() if "ttft" in k.lower()})
PY

#!/bin/bash
# Interleaved A/B of env-knob settings on ONE box: scripts/ab_env.sh <rounds> "<ENV=.. ENV=..>" "<...>" -- [bench args]
# Each setting runs bench.py once per round (settings interleaved round by round); one summary line per run.
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/benches
rounds=$1; shift
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in $(seq 1 $rounds); do
  i=0
  for s in "${sets[@]}"; do
    log=gpurun_out/benches/abenv_${r}_${i}.log
    env $s timeout -k 10 400 python -u bench.py "$@" > $log 2>&1 || { echo "FAILED: $s"; tail -20 $log; exit 3; }
    python - "$s" "$log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
keys = ["value", "p50_e2e_latency_s", "decode_device_ms_per_step", "decode_device_ms_per_step_b1",
        "explain_2k_device_ms_per_step", "explain_2k_p50_e2e_latency_s", "explain_2k_ttft_s"]
print(f"[{sys.argv[1]}]", {k: d.get(k) for k in keys if k in d}, "numerics_ok", (d.get("numerics") or {}).get("ok"))
PY
    i=$((i+1))
  done
done

#!/bin/bash
# GPU suite + default bench (+ its config-2/3 extras) + rocprof summaries of the explain (3B 2k prompt) and the
# headline 7B b32 runs.  Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/benches
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -60 gpurun_out/gpu_tests.log; exit 3; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 500 python -u bench.py > gpurun_out/benches/default.log 2>&1 || { tail -30 gpurun_out/benches/default.log; exit 4; }
tail -1 gpurun_out/benches/default.log
if [ "${PROFILE:-1}" = "1" ]; then
  bash scripts/profile_one.sh explain --model llama3.2 --batch 1 --prompt-len 2048 --new-tokens 128 --no-extras || exit 5
  bash scripts/profile_one.sh b32 --no-extras || exit 6
fi

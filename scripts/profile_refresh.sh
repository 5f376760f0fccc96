#!/bin/bash
# Fresh rocprofv3 kernel-trace + stats of the headline bench shapes; summaries under gpurun_out/prof_<tag>/
# (the big kernel_trace.csv is condensed on the box and removed so the results fit the copy-back limit)
set -o pipefail
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  bash scripts/profile_bench.sh "$tag" "$@" > gpurun_out/prof_$tag.out 2>&1 || return 1
  local d=gpurun_out/prof_$tag
  python3 scripts/prof_summary.py "$(find $d -name '*kernel_stats.csv' | head -1)" > $d/summary.txt &&
  python3 scripts/step_breakdown.py "$(find $d -name '*kernel_trace.csv' | head -1)" > $d/step_breakdown.txt 2>&1
  python3 scripts/trace_gaps.py "$(find $d -name '*kernel_trace.csv' | head -1)" > $d/gaps.txt 2>&1
  find $d -name '*kernel_trace.csv' -delete
  return 0
}
run b32 --steps 3 --warmup 1 &&
run b1 --steps 2 --warmup 1 --batch 1 &&
run explain --steps 3 --warmup 1 --batch 1 --model llama3.2 --prompt-len 2048 --new-tokens 128

#!/bin/bash
# rocprofv3 kernel traces of the latency configs (b1, 3B explain 2k) and the flagship b32.
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "b1:--batch 1" "explain:--model llama3.2 --batch 1 --prompt-len 2048" "b32:" ; do
  tag=${cfg%%:*}; args=${cfg#*:}
  bash scripts/profile_bench.sh $tag --steps 1 --warmup 1 $args > /dev/null 2>&1 || { echo "profile $tag failed"; exit 1; }
  f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
  python scripts/prof_summary.py $f > gpurun_out/prof_$tag/summary.txt
  t=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
  [ -n "$t" ] && python scripts/trace_gaps.py $t > gpurun_out/prof_$tag/gaps.txt
  echo "== $tag"; sed -n 1,14p gpurun_out/prof_$tag/summary.txt; cat gpurun_out/prof_$tag/gaps.txt
done

#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "b1:--batch 1" "explain:--model llama3.2 --batch 1 --prompt-len 2048" ; do
  tag=${cfg%%:*}; args=${cfg#*:}
  bash scripts/profile_bench.sh $tag --steps 2 --warmup 1 $args > /dev/null 2>&1 || { echo "profile $tag failed"; exit 1; }
  echo "== $tag"; python scripts/prof_summary.py gpurun_out/prof_$tag/run_kernel_stats.csv | head -14
done

#!/bin/bash
# rocprofv3 kernel trace of one bench config: scripts/profile_one.sh <tag> <bench args...>
export TMPDIR=/tmp
tag=$1; shift
bash scripts/profile_bench.sh $tag --steps 1 --warmup 1 "$@" > /dev/null 2>&1 || { echo "profile $tag failed"; exit 1; }
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f > gpurun_out/prof_$tag/summary.txt
t=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
[ -n "$t" ] && python scripts/trace_gaps.py $t > gpurun_out/prof_$tag/gaps.txt
echo "== $tag"; sed -n 1,16p gpurun_out/prof_$tag/summary.txt; cat gpurun_out/prof_$tag/gaps.txt
# the raw traces are tens of MB: keep the summaries only, so gpurun_out stays under the 64 MiB copy-back cap
find gpurun_out/prof_$tag -name "*kernel_trace.csv" -delete

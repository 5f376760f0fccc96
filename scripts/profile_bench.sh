#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run; summaries under gpurun_out/prof_<tag>/
TAG=${1:-bench}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py "$@" > gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?
tail -3 gpurun_out/prof_$TAG/bench.log
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -25 {}'
exit $rc

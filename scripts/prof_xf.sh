#!/bin/bash
# kernel stats of the 7B 300-token and 3B 2k TTFT cases with row-major (0) and fragment-major (1) prefill activations
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_xf
for v in 0 1; do
  for c in 1 0; do
    LSA_PREFILL_XF=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pxf_${v}_$c -o run -- python3 scripts/ttft_knob_ab.py none 3 $c > gpurun_out/prof_xf/run_${v}_$c.log 2>&1
    find /tmp/pxf_${v}_$c -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_xf/stats_${v}_$c.csv \;
  done
done

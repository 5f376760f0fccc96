#!/bin/bash
# rocprofv3 kernel stats of the 3B 2k prefill with the norm-free prefill on / off (scripts/ttft_nf_ab.py, one arm
# per run): scripts/prof_ttft_nf.sh -> gpurun_out/prof_nf_{nf1,nf0}/summary.txt
export TMPDIR=/tmp
for arm in nf1 nf0; do
  d=gpurun_out/prof_nf_$arm
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/ttft_nf_ab.py llama3.2 2048 $arm \
    > $d.log 2>&1 || { echo "profile $arm failed"; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 scripts/prof_summary.py $f > $d/summary.txt
  find $d -name "*kernel_trace.csv" -delete
  echo "== $arm"; sed -n 1,24p $d/summary.txt
done

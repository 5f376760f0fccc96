#!/bin/bash
# Norm-free decode at batch 32 (LSA_FUSED_NORM_MAX_B=32) vs the norm launches: 7B bf16 b32 bench A/B.
export TMPDIR=/tmp
O=gpurun_out/fn32
mkdir -p $O
for mb in 16 32; do
  LSA_FUSED_NORM_MAX_B=$mb timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_7b_fn$mb.json 2> $O/bench_7b_fn$mb.err || { tail -n 20 $O/bench_7b_fn$mb.err; exit 2; }
  cut -c1-120 $O/bench_7b_fn$mb.json
done
cd /tmp
LSA_FUSED_NORM_MAX_B=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o fn32 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -n 20 $GRAFT_REPO_ROOT/$O/prof.log; exit 3; }
echo prof ok

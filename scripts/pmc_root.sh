#!/bin/bash
# Root-cause of the round-1 `rocprofv3 --pmc` SIGSEGV in the flagship bench.
# The standalone xf GEMM repro (scripts/pmc_repro.py) profiles cleanly, so the difference is the
# bench's context: hipGraph capture.  Arm A = eager (--no-graphs), arm B = captured decode graphs.
export TMPDIR=/tmp
O=gpurun_out/pmcroot
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/eager -o p -- \
  python3 bench.py --steps 1 --warmup 1 --new-tokens 16 --no-graphs > $O/eager.log 2>&1
echo "eager rc=$?"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/graph -o p -- \
  python3 bench.py --steps 1 --warmup 1 --new-tokens 16 > $O/graph.log 2>&1
echo "graph rc=$?"

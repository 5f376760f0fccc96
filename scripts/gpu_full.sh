#!/bin/bash
# Full GPU test suite (as the driver runs it) + smoke + default bench.
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -n 5 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -n 20 $O/smoke.log; exit 2; }
tail -n 1 $O/smoke.log
timeout -k 10 200 python -u bench.py > $O/bench.log 2>&1 || { tail -n 20 $O/bench.log; exit 3; }
tail -n 1 $O/bench.log | cut -c1-300

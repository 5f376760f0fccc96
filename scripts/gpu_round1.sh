#!/bin/bash
# kernel + engine GPU tests, smoke, short bench; every GPU step under its own time limit.
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -m pytest tests/ -m gpu -q -rf -x --timeout 300 > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -30 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1
rc=$?; tail -5 gpurun_out/bench1.log; exit $rc

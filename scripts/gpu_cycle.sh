#!/bin/bash
# full GPU cycle: tests -> smoke -> bench -> rocprof stats
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -rf -x --timeout 300 > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
bash scripts/profile_bench.sh b32 --steps 2 --warmup 1 > /dev/null 2>&1
python scripts/prof_summary.py gpurun_out/prof_b32/run_kernel_stats.csv > gpurun_out/prof_b32/summary.txt; head -20 gpurun_out/prof_b32/summary.txt

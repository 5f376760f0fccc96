#!/bin/bash
# round 2, first GPU call: production-shape numerics + the --pmc SIGSEGV repro (row first, then xf)
export TMPDIR=/tmp
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests/test_prod_shapes_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2a/prod.log 2>&1
rc=$?; echo "prod rc=$rc"; case $rc in 0|1) ;; *) exit 2;; esac
timeout -k 10 120 python scripts/pmc_repro.py row 32 > gpurun_out/r2a/plain_row.log 2>&1 || exit 3
timeout -k 10 120 python scripts/pmc_repro.py xf 32 > gpurun_out/r2a/plain_xf.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r2a/pmc_row -o p -- python3 scripts/pmc_repro.py row 32 > gpurun_out/r2a/pmc_row.log 2>&1 || { echo "pmc row rc=$?"; exit 5; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r2a/pmc_xf -o p -- python3 scripts/pmc_repro.py xf 32 > gpurun_out/r2a/pmc_xf.log 2>&1 || { echo "pmc xf rc=$?"; exit 6; }
echo done

#!/bin/bash
# GPU tests only (optionally a -k filter): python -u, per-test timeout, log under gpurun_out/
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -rf -x --timeout 120 --timeout-method thread ${1:+-k "$1"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || tail -60 gpurun_out/gpu_tests.log; exit $rc

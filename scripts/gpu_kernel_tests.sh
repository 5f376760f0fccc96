#!/bin/bash
# Run the kernel numerics suite on the GPU box; output under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -rf --timeout 300 "$@" > gpurun_out/kernel_tests.log 2>&1
rc=$?
tail -40 gpurun_out/kernel_tests.log
exit $rc

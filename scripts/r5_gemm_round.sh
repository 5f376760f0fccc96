#!/bin/bash
# Round-5 prefill GEMM check on one GPU box: kernel tests, the tile-configuration sweep (-> tuning table, used by
# the engine in this same run), the GPU suite, then the default bench.  Each GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/benches
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "stream_k or gemm_silu or asymmetric or rope_epilogue" > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 600 python -u scripts/bench_prefill_gemm.py --grid --cfgs=-1,0,1,2,3,4,5,8,9,10,11,12,13 --epls 0,1 --rounds 3 \
  > gpurun_out/bench_prefill_gemm.jsonl 2> gpurun_out/bench_prefill_gemm.err || { tail -20 gpurun_out/bench_prefill_gemm.err; exit 2; }
python scripts/make_sk_tuning.py gpurun_out/bench_prefill_gemm.jsonl && cp llm_based_apache_spark_optimization_amd/ops/gemm_sk_tuning.json gpurun_out/
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -60 gpurun_out/gpu_tests.log; exit 3; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 500 python -u bench.py > gpurun_out/benches/default.log 2>&1 || { tail -30 gpurun_out/benches/default.log; exit 4; }
tail -1 gpurun_out/benches/default.log

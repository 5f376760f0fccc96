#!/bin/bash
# Round-5 GPU check: new GEMM / RoPE-epilogue / prefill-attention kernels vs their fp32 references, then the
# prefill attention A/B (one-barrier vs pipelined loop) and the stream-K epilogue A/B.  Each GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "stream_k or gemm_silu or asymmetric or rope_epilogue or attn_prefill" > gpurun_out/k_tests.log 2>&1 \
  || { tail -40 gpurun_out/k_tests.log; exit 1; }
tail -2 gpurun_out/k_tests.log
timeout -k 10 300 python -u scripts/bench_attn_prefill.py > gpurun_out/attn_prefill_pipe_ab.jsonl 2> gpurun_out/attn_prefill_pipe_ab.err \
  || { tail -20 gpurun_out/attn_prefill_pipe_ab.err; exit 2; }
cat gpurun_out/attn_prefill_pipe_ab.jsonl
timeout -k 10 400 python -u scripts/bench_prefill_gemm.py --cfgs=-1,0,8 --epls 0,1 --rounds 3 > gpurun_out/bench_epl_ab.jsonl \
  2> gpurun_out/bench_epl_ab.err || { tail -20 gpurun_out/bench_epl_ab.err; exit 3; }
echo done

#!/bin/bash
# prefill attention with V staged through VGPRs (LSA_P32_VREG=1, in-tree build) vs V by LDS-DMA (vso/vreg0.so)
export TMPDIR=/tmp
O=gpurun_out/vreg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kv_fp8_gpu.py tests/test_prod_shapes_gpu.py -k "prefill or prod" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/attn_vreg1.jsonl 2> $O/attn_vreg1.err || { tail -n 20 $O/attn_vreg1.err; exit 2; }
echo "== vreg1"; grep '^{' $O/attn_vreg1.jsonl
LSA_HIP_SO=vso/vreg0.so timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/attn_vreg0.jsonl 2> $O/attn_vreg0.err || { tail -n 20 $O/attn_vreg0.err; exit 3; }
echo "== vreg0"; grep '^{' $O/attn_vreg0.jsonl

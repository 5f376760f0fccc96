#!/bin/bash
# single-group prefill attention with the DMA 3 tiles ahead (4 buffers, LSA_P32_NBUF1=4, in-tree) vs 1 ahead
# (vso/nb2.so), and vs the paired 2-group kernel (LSA_PREFILL_PAIR auto / 0 = single)
export TMPDIR=/tmp
O=gpurun_out/nbuf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kv_fp8_gpu.py tests/test_prod_shapes_gpu.py -k "prefill or prod" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/$tag.jsonl 2> $O/$tag.err || { tail -n 20 $O/$tag.err; exit 2; }; echo "== $tag"; grep '^{' $O/$tag.jsonl | cut -c1-160; }
run pair_auto LSA_PREFILL_PAIR=auto
run single_nb4 LSA_PREFILL_PAIR=0
run single_nb2 LSA_PREFILL_PAIR=0 LSA_HIP_SO=vso/nb2.so

#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/attn5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "attn" --timeout 120 --timeout-method thread > $O/t.log 2>&1; echo "attn tests rc=$?"; grep -E "passed|failed|^E .*assert" $O/t.log | tail -n 12
LSA_PREFILL_ATTN=16 timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/pf16.jsonl 2>&1; echo "pf16 rc=$?"; grep case $O/pf16.jsonl
LSA_PREFILL_ATTN=32 timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/pf32.jsonl 2>&1; echo "pf32 rc=$?"; grep case $O/pf32.jsonl

#!/bin/bash
# KV-split prefill attention: kernel tests, then the prefill attention bench over split budgets.
export TMPDIR=/tmp
O=gpurun_out/psplit
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn_prefill" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_kv_fp8_gpu.py -k "prefill" -x -q --timeout 200 --timeout-method thread >> $O/tests.log 2>&1; rc=$?
tail -n 3 $O/tests.log
[ $rc -eq 0 ] || exit 1
for sp in 0 auto 4 6 8 10 16; do
  LSA_PREFILL_SPLIT=$sp timeout -k 10 200 python -u scripts/bench_attn_prefill.py >> $O/attn.jsonl 2> $O/attn_$sp.err || { tail -n 20 $O/attn_$sp.err; exit 2; }
done
cat $O/attn.jsonl

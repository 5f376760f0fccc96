#!/bin/bash
# fp8 KV cache (token-pair layout): tests, decode-attention microbench, 7B b32 benches bf16 / fp8 weights.
export TMPDIR=/tmp
O=gpurun_out/kv8b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kv_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "rope or attn" -x -q --timeout 200 --timeout-method thread >> $O/tests.log 2>&1; rc=$?
tail -n 5 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/bench_attn_kv8.py > $O/attn.jsonl 2> $O/attn.err || { tail -n 20 $O/attn.err; exit 2; }
cat $O/attn.jsonl
for cfg in "fp8 fp8" "bf16 fp8" "fp8 bf16"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --dtype $1 --kv-dtype $2 --steps 5 --warmup 2 > $O/bench_w$1_kv$2.json 2> $O/bench_w$1_kv$2.err || { tail -n 20 $O/bench_w$1_kv$2.err; exit 3; }
  cut -c1-300 $O/bench_w$1_kv$2.json
done

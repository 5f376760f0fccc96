#!/bin/bash
# G = 1 decode attention with 16-wave workgroups (LSA_ATTN_WV1=16) vs the 8-wave default: numerics under the
# variant, then the decode-attention bench for both builds; then the prefill KV-split sweep.
export TMPDIR=/tmp
O=gpurun_out/wv16; mkdir -p $O
LSA_HIP_SO=vso/wv16.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -k "attn or engine or graph" -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -n 30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
for v in wv8 wv16; do
  LSA_HIP_SO=vso/$v.so timeout -k 10 200 python -u scripts/bench_attn.py > $O/attn_$v.jsonl 2> $O/attn_$v.err || { tail -n 20 $O/attn_$v.err; exit 2; }
  echo "== $v"; cat $O/attn_$v.jsonl
done
LSA_HIP_SO=vso/wv16.so timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 > $O/bench_wv16.log 2>&1 || { tail -n 20 $O/bench_wv16.log; exit 3; }
tail -n 1 $O/bench_wv16.log | cut -c1-200
bash scripts/gpu_psplit.sh

#!/bin/bash
# single-buffered G = 1 decode attention over the fp8 KV cache (in-tree, LSA_ATTN_SB8=1) vs the two-set kernel
# (vso/sb8off.so): fp8-cache tests, the kv8 attention bench, the 7B fp8 + fp8-KV batch-32 bench
export TMPDIR=/tmp
O=gpurun_out/sb8; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kv_fp8_gpu.py tests/test_kernels_gpu.py -q -k "kv8 or fp8 or attn_decode" -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -n 30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
timeout -k 10 200 python -u scripts/bench_attn_kv8.py > $O/kv8_sb.jsonl 2> $O/kv8_sb.err || { tail -n 20 $O/kv8_sb.err; exit 2; }
LSA_HIP_SO=vso/sb8off.so timeout -k 10 200 python -u scripts/bench_attn_kv8.py > $O/kv8_base.jsonl 2> $O/kv8_base.err || { tail -n 20 $O/kv8_base.err; exit 3; }
echo "== sb"; cat $O/kv8_sb.jsonl; echo "== base"; cat $O/kv8_base.jsonl
for rep in 1 2; do
timeout -k 10 240 python -u bench.py --dtype fp8 --kv-dtype fp8 --steps 3 --warmup 1 > $O/b_sb_$rep.log 2>&1 || { tail -n 20 $O/b_sb_$rep.log; exit 4; }
LSA_HIP_SO=vso/sb8off.so timeout -k 10 240 python -u bench.py --dtype fp8 --kv-dtype fp8 --steps 3 --warmup 1 > $O/b_base_$rep.log 2>&1 || { tail -n 20 $O/b_base_$rep.log; exit 5; }
done
for f in $O/b_*.log; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['decode_device_ms_per_step'], d['numerics']['ok'])" $f; done

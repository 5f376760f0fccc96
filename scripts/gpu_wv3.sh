#!/bin/bash
# G = 2 / 3 decode attention with 16-wave workgroups (LSA_ATTN_WV3=16, vso/wv3_16.so) vs 8 (in-tree): numerics under
# the variant, decode-attention bench for both, then the 3B explain and 3B batch-32 benches for both
export TMPDIR=/tmp
O=gpurun_out/wv3; mkdir -p $O
LSA_HIP_SO=vso/wv3_16.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_prod_shapes_gpu.py -q -k "attn or engine or prod" -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -n 30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
timeout -k 10 200 python -u scripts/bench_attn.py > $O/attn_8.jsonl 2> $O/attn_8.err || { tail -n 20 $O/attn_8.err; exit 2; }
LSA_HIP_SO=vso/wv3_16.so timeout -k 10 200 python -u scripts/bench_attn.py > $O/attn_16.jsonl 2> $O/attn_16.err || { tail -n 20 $O/attn_16.err; exit 3; }
echo "== wv 8"; grep 3b $O/attn_8.jsonl; echo "== wv 16"; grep 3b $O/attn_16.jsonl
for v in 8 16; do
  so=""; [ $v = 16 ] && so=vso/wv3_16.so
  LSA_HIP_SO=$so timeout -k 10 240 python -u bench.py --model llama3.2 --batch 1 --prompt-len 2048 --steps 3 --warmup 1 > $O/bx_$v.log 2>&1 || { tail -n 20 $O/bx_$v.log; exit 4; }
  LSA_HIP_SO=$so timeout -k 10 240 python -u bench.py --model llama3.2 --steps 3 --warmup 1 > $O/b32_$v.log 2>&1 || { tail -n 20 $O/b32_$v.log; exit 5; }
done
for f in $O/bx_*.log $O/b32_*.log; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['decode_device_ms_per_step'], d['numerics']['ok'])" $f; done

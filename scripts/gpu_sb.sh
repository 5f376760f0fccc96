#!/bin/bash
# G = 1 decode attention single-buffered at 8 waves / SIMD (LSA_ATTN_SB=1, vso/sb1.so) vs the shipped double buffer:
# numerics under the variant, the decode-attention bench for both, then the flagship bench for both
export TMPDIR=/tmp
O=gpurun_out/sb; mkdir -p $O
LSA_HIP_SO=vso/sb1.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_prod_shapes_gpu.py -q -k "attn or engine or graph or prod" -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -n 30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
timeout -k 10 200 python -u scripts/bench_attn.py > $O/attn_base.jsonl 2> $O/attn_base.err || { tail -n 20 $O/attn_base.err; exit 2; }
LSA_HIP_SO=vso/sb1.so timeout -k 10 200 python -u scripts/bench_attn.py > $O/attn_sb1.jsonl 2> $O/attn_sb1.err || { tail -n 20 $O/attn_sb1.err; exit 3; }
echo "== base"; cat $O/attn_base.jsonl; echo "== sb1"; cat $O/attn_sb1.jsonl
for rep in 1 2; do
timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 > $O/bench_base_$rep.log 2>&1 || { tail -n 20 $O/bench_base_$rep.log; exit 4; }
LSA_HIP_SO=vso/sb1.so timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 > $O/bench_sb1_$rep.log 2>&1 || { tail -n 20 $O/bench_sb1_$rep.log; exit 5; }
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['decode_device_ms_per_step'], d['numerics']['ok'])" $f; done

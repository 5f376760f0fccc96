#!/bin/bash
# In-workgroup KV halves for prefill attention: kernel tests, then the prefill attention bench with the halves
# off / auto, then the 3B 2k explain bench (prefill of the 2k prompt runs the halves).
export TMPDIR=/tmp
O=gpurun_out/halves; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_prefill" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for hv in 0 auto; do
  LSA_PREFILL_HALVES=$hv timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/attn_$hv.jsonl 2> $O/attn_$hv.err || { tail -n 20 $O/attn_$hv.err; exit 2; }
  echo "== halves $hv"; grep '^{' $O/attn_$hv.jsonl
done
timeout -k 10 300 python -u bench.py --model llama3.2 --batch 1 --prompt-len 2048 --steps 3 --warmup 1 > $O/bench_3bx.log 2>&1 || { tail -n 20 $O/bench_3bx.log; exit 3; }
tail -n 1 $O/bench_3bx.log | cut -c1-400

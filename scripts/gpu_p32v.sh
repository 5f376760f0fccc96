#!/bin/bash
# prefill attention VALU diet (uniform group / wave ids, saddr DMA, scale folded into a packed FMA): kernel
# tests (all prefill paths incl. KV splits and halves) + the prefill attention bench + the 3B explain bench
export TMPDIR=/tmp
O=gpurun_out/p32v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kv_fp8_gpu.py tests/test_prod_shapes_gpu.py -k "prefill or prod" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 python -u scripts/bench_attn_prefill.py > $O/attn.jsonl 2> $O/attn.err || { tail -n 20 $O/attn.err; exit 2; }
grep '^{' $O/attn.jsonl
timeout -k 10 300 python -u bench.py --model llama3.2 --batch 1 --prompt-len 2048 --steps 3 --warmup 1 > $O/bench_3bx.log 2>&1 || { tail -n 20 $O/bench_3bx.log; exit 3; }
tail -n 1 $O/bench_3bx.log | cut -c1-300

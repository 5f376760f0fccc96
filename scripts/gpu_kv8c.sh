#!/bin/bash
# fp8 KV decode attention microbench (+ kernel tests) for an occupancy variant
export TMPDIR=/tmp
O=gpurun_out/kv8c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kv_fp8_gpu.py -x -q --timeout 200 --timeout-method thread -k "decode" > $O/tests.log 2>&1; rc=$?
tail -n 3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/bench_attn_kv8.py > $O/attn.jsonl 2> $O/attn.err || { tail -n 20 $O/attn.err; exit 2; }
cat $O/attn.jsonl
timeout -k 10 300 python -u bench.py --dtype fp8 --kv-dtype fp8 --steps 5 --warmup 2 > $O/bench_wfp8_kvfp8.json 2> $O/bench.err || { tail -n 20 $O/bench.err; exit 3; }
cut -c1-200 $O/bench_wfp8_kvfp8.json

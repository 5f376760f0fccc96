#!/bin/bash
# The BASELINE.json configs on one GPU; one JSON line each under gpurun_out/benches/.
mkdir -p gpurun_out/benches
run() { name=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/benches/$name.log 2>&1; rc=$?;
        tail -1 gpurun_out/benches/$name.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/benches/$name.log; exit $rc; }; }
# the default run also times BASELINE configs 2 and 3 (batch-1 and 3B 2k-explain rounds); the rest skip them
run 7b_b32_bf16 --steps 5 --warmup 2
run 7b_b1_bf16 --batch 1 --steps 3 --warmup 1 --no-extras
run 3b_explain_2k --model llama3.2 --batch 1 --prompt-len 2048 --new-tokens 128 --steps 3 --warmup 1 --no-extras
run 7b_b32_fp8 --dtype fp8 --steps 3 --warmup 1 --no-extras
run 7b_b32_fp8_kvfp8 --dtype fp8 --kv-dtype fp8 --steps 3 --warmup 1 --no-extras
run 3b_b32_bf16 --model llama3.2 --steps 3 --warmup 1 --no-extras
run 7b_b1_fp8 --dtype fp8 --batch 1 --steps 3 --warmup 1 --no-extras
run 7b_b32_mxfp4 --dtype mxfp4 --steps 3 --warmup 1 --no-extras
run 7b_b1_mxfp4 --dtype mxfp4 --batch 1 --steps 3 --warmup 1 --no-extras

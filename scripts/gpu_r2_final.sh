#!/bin/bash
# Round-2 close-out: the BASELINE bench matrix at HEAD + rocprofv3 summaries of the flagship / latency configs.
export TMPDIR=/tmp
bash scripts/bench_matrix.sh || exit 1
timeout -k 10 400 python bench.py --dtype fp8 --kv-dtype fp8 --steps 3 --warmup 1 > gpurun_out/benches/7b_b32_fp8_kvfp8.log 2>&1 || exit 2
tail -1 gpurun_out/benches/7b_b32_fp8_kvfp8.log
bash scripts/profile_one.sh fb32 || exit 3
bash scripts/profile_one.sh fx --model llama3.2 --batch 1 --prompt-len 2048 || exit 4

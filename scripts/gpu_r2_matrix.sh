#!/bin/bash
# Round-2 refresh: the BASELINE bench matrix + rocprofv3 summaries of the flagship / latency configs.
export TMPDIR=/tmp
bash scripts/bench_matrix.sh || exit 1
timeout -k 10 400 python bench.py --dtype fp8 --batch 64 --steps 3 --warmup 1 > gpurun_out/benches/7b_b64_fp8.log 2>&1 || exit 2
tail -1 gpurun_out/benches/7b_b64_fp8.log
bash scripts/profile_one.sh r2b32 || exit 3
bash scripts/profile_one.sh r2b1 --batch 1 || exit 4
bash scripts/profile_one.sh r2x --model llama3.2 --batch 1 --prompt-len 2048 || exit 5
bash scripts/profile_one.sh r2f32 --dtype fp8 || exit 6

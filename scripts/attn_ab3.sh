#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/attn3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -k "attn or engine or graph" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -n 30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
bash scripts/profile_one.sh s8x --model llama3.2 --batch 1 --prompt-len 2048 && bash scripts/profile_one.sh s8b1 --batch 1

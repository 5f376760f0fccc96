#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/attn4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_prod_shapes_gpu.py -q -k "attn or engine or graph or prod" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -n 30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
bash scripts/profile_one.sh h32 && bash scripts/profile_one.sh hb1 --batch 1 && bash scripts/profile_one.sh hx --model llama3.2 --batch 1 --prompt-len 2048 && bash scripts/profile_one.sh h3b32 --model llama3.2

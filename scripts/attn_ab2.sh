#!/bin/bash
# decode-attention A/B: kernel tests, then the bench with 8-wave vs 4-wave G=1 workgroups (+ kernel profile)
export TMPDIR=/tmp
O=gpurun_out/attn2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "attn_decode" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -n 30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
bash scripts/profile_one.sh a8 && LSA_ATTN_G1_WV=4 bash scripts/profile_one.sh a4 && bash scripts/profile_one.sh a8b1 --batch 1 && bash scripts/profile_one.sh a8x --model llama3.2 --batch 1 --prompt-len 2048

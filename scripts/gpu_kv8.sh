#!/bin/bash
# fp8 KV cache: kernel + engine tests, then the 7B b32 bench with and without the fp8 cache (bf16 and fp8 weights).
export TMPDIR=/tmp
O=gpurun_out/kv8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kv_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "rope or attn" -x -q --timeout 200 --timeout-method thread >> $O/tests.log 2>&1; rc=$?
tail -n 5 $O/tests.log
[ $rc -eq 0 ] || exit 1
for cfg in "fp8 fp8" "fp8 bf16" "bf16 fp8"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --dtype $1 --kv-dtype $2 --steps 5 --warmup 2 > $O/bench_w$1_kv$2.json 2> $O/bench_w$1_kv$2.err || { tail -n 20 $O/bench_w$1_kv$2.err; exit 2; }
  cut -c1-400 $O/bench_w$1_kv$2.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o kv8 -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp8 --kv-dtype fp8 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -n 20 $GRAFT_REPO_ROOT/$O/prof.log; exit 3; }
echo prof ok

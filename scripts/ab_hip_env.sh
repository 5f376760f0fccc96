#!/bin/bash
# HIP runtime settings vs the graph-node launch floor and the 7B b32 decode step, interleaved on one box:
# DEBUG_CLR_GRAPH_PACKET_CAPTURE (graph AQL packets recorded at instantiation) off / on.
export TMPDIR=/tmp PYTHONPATH=.
out=gpurun_out/ab_hip_env.txt
: > $out
for rep in 1 2; do
  for v in 0 1; do
    r=$(DEBUG_CLR_GRAPH_PACKET_CAPTURE=$v timeout -k 10 120 python -u scripts/probe_kernel_floor.py 2>/dev/null | tail -1) || exit 1
    echo "rep=$rep capture=$v floor $r" | tee -a $out
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extras \
      > gpurun_out/ab_hip_env_$v.log 2>&1 || { tail -20 gpurun_out/ab_hip_env_$v.log; exit 1; }
    echo "rep=$rep capture=$v b32 $(tail -1 gpurun_out/ab_hip_env_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_device_ms_per_step"])')" | tee -a $out
  done
done

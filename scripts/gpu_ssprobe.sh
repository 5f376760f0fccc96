#!/bin/bash
# timing probe: residual-epilogue row-sum atomics on one address set (shipped) vs spread over 16 (LSA_SS_SHARD_PROBE)
export TMPDIR=/tmp
O=gpurun_out/ssprobe; mkdir -p $O
timeout -k 10 300 python -u scripts/bench_res_epi.py 1,32 bf16 --rowp-only > $O/base.jsonl 2> $O/base.err || { tail -n 20 $O/base.err; exit 1; }
echo "== base"; cat $O/base.jsonl | cut -c1-260
LSA_HIP_SO=vso/ssp16.so timeout -k 10 300 python -u scripts/bench_res_epi.py 1,32 bf16 --rowp-only > $O/ssp16.jsonl 2> $O/ssp16.err || { tail -n 20 $O/ssp16.err; exit 2; }
echo "== shards 16"; cat $O/ssp16.jsonl | cut -c1-260

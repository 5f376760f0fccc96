#!/bin/bash
# rocprofv3 --pmc of the prefill GEMM (3B down, M 2048: the shape whose in-engine time exceeds its warm benchmark
# most), hand kernel vs hipBLASLt, warm vs cold caches: per-dispatch counter means under gpurun_out/pmc_cold/<tag>.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/pmc_cold
run() { tag=$1; shift; timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --stats --output-format csv -d gpurun_out/pmc_cold/$tag -o run -- python3 scripts/probe_gemm_sk.py "$@" > gpurun_out/pmc_cold/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 gpurun_out/pmc_cold/$tag.log; exit 1; }; find gpurun_out/pmc_cold/$tag -name "*kernel_trace.csv" -delete; }
SHAPE="2048 3072 8192 res -2 20"
for mode in warm cold; do
  flag=""; [ $mode = cold ] && flag="--cold"
  PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
  run sq_hand_$mode $SHAPE $flag && run sq_vendor_$mode $SHAPE $flag --vendor || exit 1
  PMC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
  run tcc_hand_$mode $SHAPE $flag && run tcc_vendor_$mode $SHAPE $flag --vendor || exit 1
done
for f in gpurun_out/pmc_cold/*.log; do echo "== $f"; grep " us," $f; done

#!/bin/bash
# rocprofv3 --pmc of the 32-row prefill attention on the 3B 2k explain shape (scripts/bench_attn_prefill.py, unsplit
# plan): two counter passes (<= 8 SQ counters each), per-dispatch means under gpurun_out/pmc_attn/<pass>.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/pmc_attn
export LSA_ATTN_CASES=3b_explain_2k LSA_ATTN_SPLITS=0
run() { tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_attn/$tag -o run -- python3 scripts/bench_attn_prefill.py > gpurun_out/pmc_attn/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 gpurun_out/pmc_attn/$tag.log; exit 1; }; find gpurun_out/pmc_attn/$tag -name "*kernel_trace.csv" -delete; }
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES && \
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE && \
python3 scripts/pmc_means.py --kernel attn_prefill32 gpurun_out/pmc_attn/sq1/ gpurun_out/pmc_attn/sq2/

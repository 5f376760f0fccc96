set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_sk
run() { tag=$1; shift; timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --stats --output-format csv -d gpurun_out/pmc_sk/$tag -o run -- python3 scripts/probe_gemm_sk.py "$@" > gpurun_out/pmc_sk/$tag.log 2>&1; find gpurun_out/pmc_sk/$tag -name "*kernel_trace.csv" -delete; }
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
run o4096_a 4096 4096 4096 bf16 0 30
run o2048_128x192_a 2048 3072 3072 bf16 12 30
PMC="SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
run o4096_b 4096 4096 4096 bf16 0 30
run o2048_128x192_b 2048 3072 3072 bf16 12 30
timeout -k 10 120 python3 scripts/probe_gemm_sk.py 4096 4096 4096 bf16 0 50
timeout -k 10 120 python3 scripts/probe_gemm_sk.py 2048 3072 3072 bf16 12 50

#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o p -- python3 scripts/gemm_pmc.py > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o p -- python3 scripts/gemm_pmc.py > /dev/null 2>&1 || exit 2
ls -R gpurun_out/pmc | head

#!/bin/bash
# SQ counter passes over plain forwards (tools/pmc_forward.py), one rocprofv3 --pmc
# invocation per counter set; summarise with tools/pmc_table.py gpurun_out/<tag>.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
export TMPDIR=/tmp
cd /tmp
O=$R/gpurun_out/$TAG
mkdir -p $O
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o p -- \
    python3 $R/tools/pmc_forward.py --out $O ${FWD_ARGS} > $O/$name.log 2>&1
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE && \
run sq3 SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL
echo rc=$?

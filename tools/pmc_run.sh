#!/bin/bash
# PMC passes over a short bench run (separate rocprofv3 invocations per counter set).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
export TMPDIR=/tmp
cd /tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$TAG/$name -o p -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-passes 1 > $R/gpurun_out/$TAG/$name.log 2>&1
}
mkdir -p $R/gpurun_out/$TAG
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INSTS_VMEM_RD && \
run fetch FETCH_SIZE && run write WRITE_SIZE
echo rc=$?

#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no trace domains) over plain forwards,
# for the shipped kernels and for one LAYER:VARIANT.  Usage: tools/pmc_ab.sh TAG LAYER:VARIANT
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmcab}
VAR=${2:-1:70}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in base var; do
  VA=""
  if [ $v = var ]; then VA="--variant $VAR"; fi
  for c in FETCH_SIZE WRITE_SIZE "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $c | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${v}_$n -o p -- \
      python3 $R/tools/pmc_forward.py --out $O/${v}_$n $VA > $O/${v}_$n.log 2>&1 || exit 1
    echo ${v}_$n ok
  done
done

# interleaved A/B of kernel variants (tools/layer_ab.py); each step under its own time limit
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/${AB_TAG:-ab}.log
: > $OUT
for spec in "$@"; do  # spec = "LAYERS:VARIANTS", e.g. "4:0,55,56"
  L=${spec%%:*}; V=${spec#*:}
  timeout -k 10 300 python -u tools/layer_ab.py --variants ${V//,/ } --layers ${L//,/ } --rounds ${AB_ROUNDS:-8} >> $OUT 2>&1 || { cat $OUT; exit 1; }
done
cat $OUT

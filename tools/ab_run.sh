set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/layer_ab.py --variants 0 55 --layers 2 3 4 --rounds 8 > gpurun_out/r03_ab_ks2.log 2>&1 && \
timeout -k 10 200 python -u tools/layer_ab.py --variants 0 56 --layers 4 --rounds 8 >> gpurun_out/r03_ab_ks2.log 2>&1
rc=$?
cat gpurun_out/r03_ab_ks2.log
exit $rc

# round-6 GPU step: fp16x3 layer2 entry with deferred stores (6:60) test + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_detector_gpu.py -q -k "entries_vgpr" --timeout 200 --timeout-method thread > $O/new_tests.log 2>&1; rc=$?; tail -2 $O/new_tests.log; [ $rc -le 1 ] || exit $rc
TAG=r06h AB_ROUNDS=8 AB_ARGS="--precision fp16x3" tools/gpu_check.sh ab:6:0,57,60

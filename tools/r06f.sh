# round-6 GPU step: shipped s2v deferred stores + x3 layer3 entry; c64v deferred-store A/B; x3 entry traces; tests; driver
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_detector_gpu.py -q -k "variants_agree or entries_vgpr or profile_and_precision" --timeout 200 --timeout-method thread > $O/new_tests.log 2>&1; rc=$?; tail -2 $O/new_tests.log; [ $rc -le 1 ] || exit $rc
TAG=r06f AB_ROUNDS=8 tools/gpu_check.sh ab:1:0,93,96 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 1 --variant 94 --launch 1 3 > $O/trace_c64v16_ds.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 6 --variant 58 --launch 5 9 --precision fp16x3 > $O/trace_x3entries.log 2>&1 || exit 1
TAG=r06f tools/gpu_check.sh test smoke driver

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06b
timeout -k 10 300 python3 -u -m pytest tests/test_detector_gpu.py -x -q -k "s2k or variants_agree" --timeout 200 --timeout-method thread > gpurun_out/r06b/s2k_test.log 2>&1; rc=$?; tail -3 gpurun_out/r06b/s2k_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 6 --variant 56 --launch 9 13 > gpurun_out/r06b/trace_s2k.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 6 --variant 49 --launch 5 > gpurun_out/r06b/trace_s2v.log 2>&1 || exit 1
TAG=r06b AB_ROUNDS=6 tools/gpu_check.sh ab:6:0,55,48,40 test smoke driver

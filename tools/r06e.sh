# round-6 GPU step: new fp16x3 layer2 entry + tick test, A/B, c64v / s2v traces, full tests, driver command
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_detector_gpu.py tests/test_pose_tick_split_gpu.py -q -k "more_trajectories or entries_vgpr" --timeout 200 --timeout-method thread > $O/new_tests.log 2>&1; rc=$?; tail -2 $O/new_tests.log; [ $rc -le 1 ] || exit $rc  # (assertion failures: go on; a fault or a timeout: stop)
TAG=r06e AB_ROUNDS=6 AB_ARGS="--precision fp16x3" tools/gpu_check.sh ab:6:0,57 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 1 --variant 84 --launch 1 3 > $O/trace_c64v16.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 1 --variant 86 --launch 2 4 > $O/trace_c64v8.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 6 --variant 54 --launch 5 > $O/trace_s2v_ds.log 2>&1 || exit 1
mv $O/ab.log $O/ab_x3.log
TAG=r06e AB_ROUNDS=8 tools/gpu_check.sh ab:6:0,52,53 test smoke driver

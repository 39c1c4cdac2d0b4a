# round-6 GPU step: pose-tick test fix, s2v deferred-store A/B, c64v traces, full tests, driver command
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_pose_tick_split_gpu.py -x -q -k "more_trajectories" --timeout 200 --timeout-method thread > $O/tick_test.log 2>&1; rc=$?; tail -2 $O/tick_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 1 --variant 84 --launch 1 3 > $O/trace_c64v16.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 1 --variant 86 --launch 2 4 > $O/trace_c64v8.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/trace_launch.py --layer 6 --variant 54 --launch 5 > $O/trace_s2v_ds.log 2>&1 || exit 1
TAG=r06c AB_ROUNDS=8 tools/gpu_check.sh ab:6:0,52,53 test smoke driver

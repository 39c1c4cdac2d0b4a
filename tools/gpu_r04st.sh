# round 4: split tick -- vs fused at every L, 1000-tick stress of the split and fused forms
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04st}
mkdir -p $out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pose_tick_split_gpu.py > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
TICK_SPLIT=1 TICK_L=24 TICK_N=1000 timeout -k 10 120 python3 -u tools/tick_stress.py > $out/stress_split24.log 2>&1
rc=$?; echo "stress split L=24 rc=$rc"; tail -1 $out/stress_split24.log; [ $rc -eq 0 ] || exit $rc
TICK_SPLIT=1 TICK_L=7 TICK_N=1000 timeout -k 10 120 python3 -u tools/tick_stress.py > $out/stress_split7.log 2>&1
rc=$?; echo "stress split L=7 rc=$rc"; tail -1 $out/stress_split7.log; exit $rc

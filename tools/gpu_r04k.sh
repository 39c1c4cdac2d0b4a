# round 4: cyclic-reduction GN step (paired assembly) -- parity tests, A/B per T, phase trace at T = 3
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04k}
mkdir -p $out
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gn_gpu.py tests/test_gn_kp_gpu.py tests/test_streaming_pose_gpu.py > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gn_ab.py --na 128 64 --T 1000 512 256 64 3 --rounds 5 > $out/gn_cr_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $out/gn_cr_ab.log; [ $rc -eq 0 ] || exit $rc
GN_TRACE=1 GN_VARIANT=64 timeout -k 10 120 python3 tools/gn_ab.py > $out/cr_trace.log 2>&1
rc=$?; cat $out/cr_trace.log; exit $rc

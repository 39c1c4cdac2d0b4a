# round 4: cyclic-reduction GN step -- parity tests, then the A/B against the two-ended kernel per T
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04i}
mkdir -p $out
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gn_gpu.py tests/test_gn_kp_gpu.py tests/test_streaming_pose_gpu.py > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/gn_ab.py --na 128 64 --T 1000 512 256 128 64 32 16 3 --rounds 5 > $out/gn_cr_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $out/gn_cr_ab.log; exit $rc

# round 4: fp16x3 role-split stem -- bit-identity tests, then the one-process A/B against the all-waves form
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04l}
mkdir -p $out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_detector_gpu.py -k "fp16x3" > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/layer_ab.py --precision fp16x3 --variants 0 30 --layers 0 --rounds 6 > $out/stem_x3_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $out/stem_x3_ab.log; exit $rc

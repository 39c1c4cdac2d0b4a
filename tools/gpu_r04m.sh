# round 4: fp16x3 role-split stem and layer4's image-pair s2w entry -- tests, then one-process A/Bs
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04m}
mkdir -p $out
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_detector_gpu.py -k "fp16x3 or variants or invariance" > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/layer_ab.py --precision fp16x3 --variants 0 30 --layers 0 --rounds 5 > $out/stem_x3_ab.log 2>&1
rc=$?; echo "stem ab rc=$rc"; tail -22 $out/stem_x3_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/layer_ab.py --variants 0 48 49 --layers 6 --rounds 8 > $out/l4_s2w_ab.log 2>&1
rc=$?; echo "l4 ab rc=$rc"; tail -22 $out/l4_s2w_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/layer_ab.py --precision fp16x3 --variants 0 48 --layers 6 --rounds 5 > $out/l4_s2w_x3_ab.log 2>&1
rc=$?; echo "l4 x3 ab rc=$rc"; tail -22 $out/l4_s2w_x3_ab.log; exit $rc

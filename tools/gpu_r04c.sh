# round 4: s2w stride-2 entries -- A/B against conv_s2x, then the detector / streaming tests
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r04c}
mkdir -p $out
timeout -k 10 300 python -u tools/layer_ab.py --variants 0 10 41 42 --layers 6 --rounds 8 > $out/s2w_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v -rA --timeout 120 --timeout-method thread tests/test_detector_gpu.py tests/test_streaming_pose_gpu.py tests/test_streaming_gpu.py tests/test_gn_gpu.py -m gpu > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; exit $rc

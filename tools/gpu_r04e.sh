# round 4: fp16x3 row-split entries -- A/B against conv_s2x X3, then the detector tests
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r04e}
mkdir -p $out
timeout -k 10 300 python -u tools/layer_ab.py --precision fp16x3 --variants 0 45 46 --layers 6 --rounds 6 > $out/x3_entry_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v -rA --timeout 120 --timeout-method thread tests/test_detector_gpu.py tests/test_streaming_gpu.py -m gpu > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; exit $rc

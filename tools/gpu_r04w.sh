# round 4: latency-mode small tiles -- parity tests (factors / GN / window / streaming), tick timing + trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04w}
mkdir -p $out
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_detector_gpu.py tests/test_streaming_pose_gpu.py tests/test_pipeline_gpu.py tests/test_streaming_gpu.py > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 python3 $R/tools/streaming_bench.py --ticks 100 > $out/streaming_plain.jsonl 2>&1
rc=$?; echo "plain rc=$rc"; tail -1 $out/streaming_plain.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $R/tools/streaming_bench.py --ticks 100 > $out/streaming_kt.jsonl 2>&1
rc=$?; echo "kt rc=$rc"; exit $rc

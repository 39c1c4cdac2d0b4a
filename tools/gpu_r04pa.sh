# round 4: pre-ahead pose tick -- pose tests, streaming bench (pose / pose_parity / _ahead modes)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04pa}
mkdir -p $out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_streaming_pose_gpu.py tests/test_streaming_gpu.py > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 python3 $R/tools/streaming_bench.py --ticks 100 > $out/streaming.jsonl 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.loads(open('$out/streaming.jsonl').read().strip().split(chr(10))[-1])
for k,v in d.items():
    if isinstance(v, dict): print(k, v.get('p50_ms'), v.get('p99_ms'), v.get('device_ms_per_tick'), v.get('latency_path_ms'))"

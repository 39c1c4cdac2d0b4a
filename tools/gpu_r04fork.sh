# round 4: split pose tick -- fork/join placement A/B (PA_TICK_FORK 0: pre on a side stream, 2: forward on
# the side stream, 3: 2 without the pre half (timing only), 4: serial, 9: unsplit), tick device time
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04fork}
mkdir -p $out
cd $R
PA_TICK_FORK=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_streaming_pose_gpu.py > $out/tests2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $out/tests2.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
for m in ${MODES:-9 2 3 4 0 9 2 3 4 0}; do
  PA_TICK_FORK=$m timeout -k 10 200 python3 $R/tools/streaming_bench.py --ticks 100 > $out/fork$m.jsonl 2>&1 || exit 1
  python3 -c "
import json,sys; d=json.loads(open('$out/fork$m.jsonl').read().strip().split(chr(10))[-1])
print('mode $m', d['pose']['device_ms_per_tick'], d['pose_parity']['device_ms_per_tick'], d['pose']['p50_ms'], d['pose_parity']['p50_ms'])"
done

# round 4: zero-copy tick input (the stem / preprocess read the pinned staging) -- A/B of the tick, equality check
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04v}
mkdir -p $out
cd /tmp
timeout -k 10 120 python3 -u $R/tools/zero_copy_check.py > $out/check.log 2>&1
rc=$?; echo "check rc=$rc"; tail -3 $out/check.log; [ $rc -eq 0 ] || exit $rc
for z in "" "--zero-copy" "" "--zero-copy"; do
  timeout -k 10 200 python3 $R/tools/streaming_bench.py --ticks 100 $z >> $out/ab.jsonl 2>/dev/null || exit 1
done
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print({k: (v['p50_ms'], v['device_ms_per_tick']) for k, v in d.items() if isinstance(v, dict)})
"

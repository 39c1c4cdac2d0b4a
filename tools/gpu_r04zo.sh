# round 4: zero-copy output A/B (streaming bench, --zero-copy-out 1 / 0 interleaved)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04zo}
mkdir -p $out
cd /tmp
for z in 1 0 1 0; do
  timeout -k 10 200 python3 $R/tools/streaming_bench.py --ticks 100 --zero-copy-out $z > $out/zo$z.jsonl 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$out/zo$z.jsonl').read().strip().split(chr(10))[-1])
print('zc_out $z', ' '.join(f'{k}:{v.get(\"p50_ms\")}/{v.get(\"device_ms_per_tick\")}/{v.get(\"latency_path_ms\")}' for k,v in d.items() if isinstance(v, dict)))"
done

# round 4: stream priority A/B for the split tick (PA_PRIO 0 / 1 forward stream high / 2 tick stream high;
# the PA_PRIO switch was a temporary patch of streaming.py, not kept: DESIGN.md Appendix D)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04prio}
mkdir -p $out
cd /tmp
for z in 0 1 2 0 1 2; do
  PA_PRIO=$z timeout -k 10 200 python3 $R/tools/streaming_bench.py --ticks 60 > $out/prio$z.jsonl 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$out/prio$z.jsonl').read().strip().split(chr(10))[-1])
print('prio $z', ' '.join(f'{k}:{v.get(\"p50_ms\")}/{v.get(\"device_ms_per_tick\")}/{v.get(\"latency_path_ms\")}' for k,v in d.items() if isinstance(v, dict)))"
done

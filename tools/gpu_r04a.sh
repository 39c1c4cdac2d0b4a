# round-4 GPU check: the whole -m gpu suite, then the driver's bench command
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r04a}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v -rA --timeout 120 --timeout-method thread tests -m gpu > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; exit $rc

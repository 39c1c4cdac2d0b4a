# round 4: split-K reduces with compile-time split counts -- bit identity, per-launch A/B at B = 3, streaming ticks
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${TAG:-r04r}
mkdir -p $out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_detector_gpu.py -k "split_k" > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/layer_ab.py --batch 3 --split-k 8 --variants 0 5 --layers 7 --rounds 6 > $out/reduce_ab_fp16.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -30 $out/reduce_ab_fp16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/layer_ab.py --batch 3 --split-k 8 --precision fp16x3 --variants 0 5 --layers 7 --rounds 6 > $out/reduce_ab_x3.log 2>&1
rc=$?; echo "ab x3 rc=$rc"; tail -3 $out/reduce_ab_x3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/streaming_bench.py --ticks 100 > $out/streaming.jsonl 2>&1
rc=$?; echo "streaming rc=$rc"; tail -1 $out/streaming.jsonl; exit $rc

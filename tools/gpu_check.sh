#!/bin/bash
# GPU-box check: gpu tests, then a short bench.  Stops at the first fault/timeout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-500} python -m pytest tests -m gpu -q -rA -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo pytest_rc=$rc
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo bench_rc=$rc
tail -1 gpurun_out/bench.log
exit $rc

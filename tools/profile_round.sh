#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace --stats of the bench command
# itself, kernel traces of plain forwards (fp16 and the fp16x3 parity mode) and of the
# factor path, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes over fp16
# forwards (no trace domains combined with --pmc).  Summarise afterwards on the host
# with tools/rocprof_summary.py --dir gpurun_out/<tag> --tag <tag>.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
BENCH_ARGS=${BENCH_ARGS:-}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_kt -o kt -- \
  python3 $R/bench.py $BENCH_ARGS > $O/bench.log 2>&1 && echo bench_kt_ok && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/fwd_kt -o kt -- \
  python3 $R/tools/pmc_forward.py --out $O > $O/fwd_kt.log 2>&1 && echo fwd_kt_ok && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x3_kt -o kt -- \
  python3 $R/tools/pmc_forward.py --precision fp16x3 --out $O/x3 > $O/x3_kt.log 2>&1 && echo x3_kt_ok && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fac_kt -o kt -- \
  python3 $R/tools/factor_prof.py > $O/fac_kt.log 2>&1 && echo fac_kt_ok && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- \
  python3 $R/tools/pmc_forward.py --out $O > $O/fetch.log 2>&1 && echo fetch_ok && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- \
  python3 $R/tools/pmc_forward.py --out $O > $O/write.log 2>&1 && echo write_ok
rc=$?
tail -1 $O/bench.log
exit $rc

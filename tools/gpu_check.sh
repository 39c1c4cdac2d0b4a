#!/bin/bash
# The one GPU-box runner:  gpurun -- 'TAG=r05x tools/gpu_check.sh STEP [STEP ...]'
# Every step runs under its own time limit; the first failing step ends the call (no retries,
# nothing else touches the GPU after a fault or a timeout).  Output goes to gpurun_out/$TAG/.
#
#   test            python -m pytest tests -m gpu  ($PYTEST_ARGS, e.g. "-k streaming")
#   smoke           __graft_entry__.smoke()
#   bench           python bench.py $BENCH_ARGS            -> bench.jsonl (default: the full bench)
#   driver          python bench.py --gpus 1 --steps 20 --warmup 5 (the driver's own command)
#   ab:L,L:V,V      interleaved per-launch A/B in one process (tools/layer_ab.py), layers L, variants V
#                   ($AB_ROUNDS rounds, $AB_ARGS extra, e.g. "--precision fp16x3")
#   fwdab:L:V[,..]  interleaved whole-forward A/B (tools/head_ab.py --ab L:V ...)
#   benchab:L:V[,L:V] the driver's bench command, shipped and with the variants
#                   (PERSEUS_AMD_BENCH_VARIANTS), alternated $BENCHAB_PAIRS times -> benchab.jsonl
#   benchabx3:L:V   the same for the parity-mode models (PERSEUS_AMD_BENCH_VARIANTS_PARITY)
#   soab:A.so[,B.so] interleaved A/B of other builds of the library against the in-tree one
#                   (tools/so_ab.py: one process per build and round; PERSEUS_AMD_LIB_AB)
#   profile         rocprofv3 --kernel-trace --stats of the bench command + kernel traces of plain
#                   fp16 / fp16x3 forwards + the factor path + FETCH_SIZE and WRITE_SIZE passes
#                   (summarise here: tools/rocprof_summary.py --dir gpurun_out/$TAG --tag $TAG)
#   fetch[:name]    FETCH_SIZE + WRITE_SIZE passes only (over pmc_forward.py $FWD_ARGS) -> name_fetch/, name_write/
#   mfma            MFMA counter pass (summarise: tools/mfma_counters.py gpurun_out/$TAG --tag $TAG)
#   sq              three SQ counter passes (summarise: tools/pmc_table.py gpurun_out/$TAG)
#   stream          streaming bench (tools/streaming_bench.py $STREAM_ARGS)
#   stress          1,000 back-to-back pose ticks (tools/tick_stress.py)
# $FWD_ARGS is passed to tools/pmc_forward.py (e.g. "--variant 1:5").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${TAG:-check}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
PY="python3 -u"

pmc() {  # name, counters...  (one --pmc group per run, no trace domains)
  local name=$1; shift
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o p -- \
    $PY $R/tools/pmc_forward.py --out $O ${FWD_ARGS}) > $O/$name.log 2>&1
}

step() {
  local s=$1
  case $s in
    test)
      (cd $R && timeout -k 10 ${TEST_TIMEOUT:-900} $PY -m pytest tests -m gpu -x -q -rf --timeout 300 \
        --timeout-method thread ${PYTEST_ARGS}) > $O/pytest_gpu.log 2>&1
      local rc=$?; tail -3 $O/pytest_gpu.log; return $rc ;;
    smoke)
      (cd $R && timeout -k 10 300 $PY -c "import __graft_entry__ as g; g.smoke()") > $O/smoke.log 2>&1
      local rc=$?; tail -4 $O/smoke.log; return $rc ;;
    bench)
      (cd $R && timeout -k 10 ${BENCH_TIMEOUT:-500} $PY bench.py ${BENCH_ARGS}) > $O/bench.jsonl 2>$O/bench.err
      local rc=$?; tail -c 600 $O/bench.jsonl; return $rc ;;
    driver)
      (cd $R && timeout -k 10 500 $PY bench.py --gpus 1 --steps 20 --warmup 5) > $O/bench_driver_cmd.jsonl \
        2>$O/bench_driver_cmd.err
      local rc=$?; tail -c 300 $O/bench_driver_cmd.jsonl; return $rc ;;
    ab:*)
      local spec=${s#ab:}; local L=${spec%%:*}; local V=${spec#*:}
      (cd $R && timeout -k 10 300 $PY tools/layer_ab.py --variants ${V//,/ } --layers ${L//,/ } \
        --rounds ${AB_ROUNDS:-8} ${AB_ARGS}) >> $O/ab.log 2>&1
      local rc=$?; tail -4 $O/ab.log; return $rc ;;
    soab:*)  # soab:OLD.so[,OLD2.so]: the in-tree build against other builds (tools/so_ab.py)
      local libs=${s#soab:}
      (cd $R && timeout -k 10 900 $PY tools/so_ab.py ${libs//,/ } perseus_amd/lib/libperseus_amd.so \
        --rounds ${AB_ROUNDS:-6} ${AB_ARGS}) >> $O/soab.log 2>&1
      local rc=$?; tail -25 $O/soab.log; return $rc ;;
    fwdab:*)
      local spec=${s#fwdab:}
      (cd $R && timeout -k 10 400 $PY tools/head_ab.py --ab ${spec//,/ } ${AB_ARGS}) >> $O/fwdab.log 2>&1
      local rc=$?; tail -4 $O/fwdab.log; return $rc ;;
    benchab:*|benchabx3:*)
      local vs=${s#benchab:}; local ev=PERSEUS_AMD_BENCH_VARIANTS
      if [[ $s == benchabx3:* ]]; then vs=${s#benchabx3:}; ev=PERSEUS_AMD_BENCH_VARIANTS_PARITY; fi
      for k in $(seq ${BENCHAB_PAIRS:-2}); do
        (cd $R && timeout -k 10 400 $PY bench.py --gpus 1 --steps 20 --warmup 5 --no-streaming) 2>>$O/benchab.err | \
          sed 's/^/{"ab": "shipped", "line": /; s/$/}/' >> $O/benchab.jsonl || return 1
        (cd $R && env $ev=$vs timeout -k 10 400 $PY bench.py --gpus 1 --steps 20 --warmup 5 \
          --no-streaming) 2>>$O/benchab.err | sed "s/^/{\"ab\": \"$vs\", \"line\": /; s/\$/}/" >> $O/benchab.jsonl || return 1
        echo "pair $k done"
      done ;;
    profile)
      (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_kt -o kt -- \
        $PY $R/bench.py ${BENCH_ARGS}) > $O/bench.log 2>&1 && echo bench_kt_ok && \
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/fwd_kt -o kt -- \
        $PY $R/tools/pmc_forward.py --out $O ${FWD_ARGS}) > $O/fwd_kt.log 2>&1 && echo fwd_kt_ok && \
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x3_kt -o kt -- \
        $PY $R/tools/pmc_forward.py --precision fp16x3 --out $O/x3) > $O/x3_kt.log 2>&1 && echo x3_kt_ok && \
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fac_kt -o kt -- \
        $PY $R/tools/factor_prof.py) > $O/fac_kt.log 2>&1 && echo fac_kt_ok && \
      pmc fetch FETCH_SIZE && echo fetch_ok && pmc write WRITE_SIZE && echo write_ok ;;
    fetch|fetch:*)
      local nm=${s#fetch}; nm=${nm#:}
      pmc ${nm:+${nm}_}fetch FETCH_SIZE && pmc ${nm:+${nm}_}write WRITE_SIZE && echo fetch_ok ;;
    mfma)
      pmc mfma SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE && echo mfma_ok ;;
    sq)
      pmc sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
        GRBM_GUI_ACTIVE && \
      pmc sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD \
        SQ_WAVES GRBM_GUI_ACTIVE && \
      pmc sq3 SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD \
        SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL && echo sq_ok ;;
    stream)
      (cd $R && timeout -k 10 300 $PY tools/streaming_bench.py ${STREAM_ARGS}) > $O/stream.jsonl 2>&1
      local rc=$?; tail -2 $O/stream.jsonl; return $rc ;;
    stress)
      (cd $R && timeout -k 10 300 $PY tools/tick_stress.py) > $O/stress.log 2>&1
      local rc=$?; tail -3 $O/stress.log; return $rc ;;
    *) echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  echo "== $s"
  step "$s" || { rc=$?; echo "step $s failed rc=$rc"; exit $rc; }
done
echo all_ok

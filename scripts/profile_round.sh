#!/bin/bash
# Profile the default bench workload on the GPU box:
#   1. rocprofv3 --kernel-trace --stats (per-kernel durations)
#   2. PMC passes, each counter group in its own run (never combined with trace domains):
#      SQ issue counters, FETCH_SIZE, WRITE_SIZE
#   3. the FETCH_SIZE / WRITE_SIZE calibration (scripts/ubench/fetch_calib) on known byte counts
# then summarise into gpurun_out/$TAG/ (copy what is to be committed into profiles/).
# usage: [PROF_CONFIG=5m_1080p] scripts/profile_round.sh TAG
set -u
TAG=${1:-prof}
CFG=${PROF_CONFIG:-1m_1080p}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
BENCH="python3 $R/bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline"
PBENCH="python3 $R/bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-stage-events"
CAL=$R/scripts/ubench/fetch_calib
step() {
  echo "=== $*"
  "$@"
  rc=$?
  echo "=== rc=$rc"
  return $rc
}
step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $BENCH > $OUT/trace.log 2>&1 && \
step timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/sq1 -o sq1 --output-format csv -- $PBENCH > $OUT/sq1.log 2>&1 && \
step timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/sq2 -o sq2 --output-format csv -- $PBENCH > $OUT/sq2.log 2>&1 && \
step timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- $PBENCH > $OUT/fetch.log 2>&1 && \
step timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- $PBENCH > $OUT/write.log 2>&1 && \
step timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/cal_fetch -o cal_fetch --output-format csv -- $CAL > $OUT/cal_fetch.log 2>&1 && \
step timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $OUT/cal_write -o cal_write --output-format csv -- $CAL > $OUT/cal_write.log 2>&1
rc=$?
STAMP=$(cat $R/3d_gaussian_splatting_amd/lib/libgsr_hip.so.stamp)
python3 $R/scripts/pmc_summary.py $OUT/sq1 $OUT/sq2 $OUT/fetch $OUT/write --calib $OUT/cal_fetch $OUT/cal_write \
  --lib-stamp $STAMP --workload $CFG --traffic $OUT/pmc_traffic.json > $OUT/pmc_summary.txt 2>&1
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
exit $rc

#!/bin/bash
# rocprofv3 PMC passes over a short bench run (each counter group in its own pass; no
# trace domains combined with --pmc).  Output: gpurun_out/pmc/<tag>_*.csv
set -u
cd /tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
BENCH="python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage-events"
pass() {
  tag=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d $OUT/$tag -o $tag --output-format csv -- $BENCH > $OUT/$tag.log 2>&1
  rc=$?; echo "pass $tag rc=$rc"; return $rc
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE

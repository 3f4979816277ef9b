#!/bin/bash
# SQ issue counters of the blend kernels for several kernel variants (one rocprofv3 PMC pass
# per variant; no trace domains).  usage: scripts/pmc_variants.sh VARNAME v1 v2 ...
set -u
R=$GRAFT_REPO_ROOT
VAR=$1; shift
OUT=$R/gpurun_out/pmcvar
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for v in "$@"; do
  export $VAR=$v
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    -d $OUT/$VAR$v -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage-events > $OUT/$VAR$v.log 2>&1
  rc=$?
  echo "$VAR=$v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 $R/scripts/pmc_summary.py $OUT/$VAR$v | grep -E "kernel|blend" | cut -c1-400
done

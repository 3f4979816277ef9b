#!/bin/bash
# One rocprofv3 PMC pass (SQ issue counters) of a command per environment setting.
# usage: scripts/pmc_env.sh OUTTAG "ENV1=a ENV2=b" "ENV1=c" -- python3 script.py args...
set -u
R=$GRAFT_REPO_ROOT
TAG=$1; shift
SETS=()
while [ "$1" != "--" ]; do SETS+=("$1"); shift; done
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
for s in "${SETS[@]}"; do
  for kv in $s; do export "$kv"; done
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -d $OUT/v$i -o p --output-format csv -- "$@" > $OUT/v$i.log 2>&1
  rc=$?
  echo "== [$s] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 $R/scripts/pmc_summary.py $OUT/v$i | grep -E "^kernel|blend" | cut -c1-300
  i=$((i+1))
done

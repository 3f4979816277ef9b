#!/bin/bash
# WRITE_SIZE of every kernel for the in-tree library and each lib/variants/<name> build (one
# rocprofv3 --pmc pass per library, nothing else collected), summarised per variant.
# usage: scripts/variant_writes.sh TAG name1 [name2 ...]
set -u
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for v in base "$@"; do
  LIBARG=""
  [ "$v" != base ] && LIBARG="--lib $R/3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so"
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_$v -o w --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage-events $LIBARG > $OUT/w_$v.log 2>&1 || exit $?
  echo "=== $v" >> $OUT/writes.txt
  python3 $R/scripts/pmc_summary.py $OUT/w_$v >> $OUT/writes.txt 2>&1
done

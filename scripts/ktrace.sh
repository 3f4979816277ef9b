#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of one command; the stats CSV lands in
# gpurun_out/TAG/NAME_kernel_stats.csv.   usage: scripts/ktrace.sh TAG NAME -- python3 args...
set -u
TAG=$1; NAME=$2; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_$NAME -o trace --output-format csv -- "$@" > $O/trace_$NAME.log 2>&1
rc=$?
find $O/trace_$NAME -name "*kernel_stats.csv" -exec cp {} $O/${NAME}_kernel_stats.csv \;
exit $rc

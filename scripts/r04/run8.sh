#!/bin/bash
# round 4, GPU call 8: the whole -m gpu suite as the driver runs it
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_8
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 1150 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1

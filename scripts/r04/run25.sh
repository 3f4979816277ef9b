#!/bin/bash
# round 4, GPU call 25: the whole -m gpu suite, smoke() and the bench line at the final HEAD
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_25
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err

#!/bin/bash
# round 4, GPU call 24: the configs[4] bench line at the final library (C++ loop, 30k iterations,
# 6M initial points, 48 views at 1280x832 of an 8M-Gaussian ground truth)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_24
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --mode loop --loop-gt 8000000 --loop-init 6000000 --loop-views 48 --iters 30000 > $O/bench_loop30k.json 2> $O/bench_loop30k.err

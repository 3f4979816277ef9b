#!/bin/bash
# kernel trace of the training-step bench (bench.py --mode train) -> gpurun_out/train_trace
set -u
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/train_trace -o t --output-format csv -- python3 $R/bench.py --mode train --steps 20 --warmup 5 > $R/gpurun_out/train_trace.log 2>&1

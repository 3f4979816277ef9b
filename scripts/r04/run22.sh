#!/bin/bash
# round 4, GPU call 22: moving cameras on the multi-GPU step -- set_camera + rebalance_every in
# the Python (two processes) and C++ (RCCL world 1, graph) ShardStep, with the other shard tests
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_22
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py tests/test_gpu_shard_cpp.py tests/test_gpu_dist.py > $O/shard_tests.log 2>&1

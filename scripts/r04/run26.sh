#!/bin/bash
# round 4, GPU call 26: the Python ShardStep's agreed overflow check (every rank's words in the
# image all-gather footer, checked `lag` steps later) -- the multi-process and shard tests
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_26
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py tests/test_gpu_dist.py tests/test_gpu_shard_cpp.py tests/test_gpu_parity.py -k "multiproc or two_process or dist or shard or rccl or overflow" > $O/shard_tests.log 2>&1

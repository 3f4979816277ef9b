#!/bin/bash
# round 4, GPU call 23: host time per step of the multi-GPU step, Python ShardStep and the C++
# graph-replayed one, against its GPU time (world 1; 1M and 5M)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_23
mkdir -p $O
cd $R
export TMPDIR=/tmp
for c in 1m_1080p 5m_1080p; do
  timeout -k 10 200 python scripts/shard_host_time.py --config $c --impl cpp >> $O/host_time.jsonl 2>> $O/host_time.err || exit $?
  timeout -k 10 200 python scripts/shard_host_time.py --config $c >> $O/host_time.jsonl 2>> $O/host_time.err || exit $?
done

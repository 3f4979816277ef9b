#!/bin/bash
# round 4, GPU call 11: the multi-GPU rehearsal with the end-of-round library
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_11
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python scripts/band_sim.py --config 1m_1080p --worlds 1,2,4,8 > $O/band_sim_1m.jsonl 2> $O/band_sim_1m.err && \
timeout -k 10 400 python scripts/band_sim.py --config 5m_1080p --worlds 1,2,4,8 > $O/band_sim_5m.jsonl 2> $O/band_sim_5m.err

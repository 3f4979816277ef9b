#!/bin/bash
# round 4, GPU call 4: the 5M multi-GPU rehearsal and the splat-pack A/B at the N = 8 shapes
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_4
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python scripts/band_sim.py --config 5m_1080p --worlds 1,8 > $O/band_sim_5m.jsonl 2> $O/band_sim_5m.err && \
timeout -k 10 600 bash scripts/band_ab.sh $O/band_ab_1m.jsonl 2 1m_1080p 8 packold pack1 pack2 && \
timeout -k 10 600 bash scripts/band_ab.sh $O/band_ab_5m.jsonl 2 5m_1080p 8 packold pack1

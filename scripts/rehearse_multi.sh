#!/bin/bash
# Multi-rank rehearsal on ONE GPU: every rank's compute of the N-GPU path (band_sim, no
# collectives) for world 1/2/4/8 at 1M and 5M Gaussians, then the full bench path with gloo
# at 2 and 4 ranks sharing the card (exchange code under real process groups).
# usage: scripts/rehearse_multi.sh OUTDIR
set -u
OUT=${1:-gpurun_out/rehearse}
mkdir -p $OUT
for cfg in 1m_1080p 5m_1080p; do
  timeout -k 10 240 python3 scripts/band_sim.py --config $cfg --steps 5 >> $OUT/band_sim.jsonl 2>>$OUT/band_sim.err || exit $?
done
for w in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29500 + w)) bench.py --gpus $w --steps 5 --warmup 2 --dist-backend gloo \
    > $OUT/gloo_$w.log 2>&1 || exit $?
done

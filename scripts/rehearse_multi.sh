#!/bin/bash
# Multi-rank rehearsal on ONE GPU: per-rank band compute (band_sim, no collectives) for
# world 2/4/8, then the full bench path with gloo at 2, 4 and 8 ranks sharing the card.
# usage: scripts/rehearse_multi.sh OUTDIR
set -u
OUT=${1:-gpurun_out/rehearse}
mkdir -p $OUT
for w in 2 4 8; do
  for r in $(seq 0 $((w-1))); do
    timeout -k 10 120 python3 scripts/band_sim.py --world $w --rank $r --steps 10 --warmup 3 >> $OUT/band_sim.jsonl 2>>$OUT/band_sim.err || exit $?
  done
done
for w in 2 4 8; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29500 + w)) bench.py --gpus $w --steps 5 --warmup 2 --dist-backend gloo \
    > $OUT/gloo_$w.log 2>&1 || exit $?
done

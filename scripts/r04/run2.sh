#!/bin/bash
# round 4, GPU call 2: multi-GPU rehearsal at HEAD (B2 band sum fused, presort in bands) and the
# splat-pack block size A/B at the 1M / 5M N = 8 shapes
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_2
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_train_loop.py -k configs4 \
  > $O/tests_configs4.log 2>&1 ; r=$?; [ $r -le 1 ] && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_multiproc.py tests/test_gpu_shard_cpp.py \
  > $O/tests_shard.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "shard" > $O/tests_shard_parity.log 2>&1 && \
timeout -k 10 300 python scripts/band_sim.py --config 1m_1080p --worlds 1,2,4,8 > $O/band_sim_1m.jsonl 2> $O/band_sim_1m.err && \
timeout -k 10 400 python scripts/band_sim.py --config 5m_1080p --worlds 1,8 > $O/band_sim_5m.jsonl 2> $O/band_sim_5m.err && \
timeout -k 10 600 bash scripts/band_ab.sh $O/band_ab_1m.jsonl 2 1m_1080p 8 packold pack1 pack2 && \
timeout -k 10 600 bash scripts/band_ab.sh $O/band_ab_5m.jsonl 2 5m_1080p 8 packold pack1

#!/bin/bash
# round 4, GPU call 21: the multi-GPU rehearsal and the views benches with the final library, then
# call 22's shard tests (moving cameras: set_camera + rebalance_every)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_21
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python scripts/band_sim.py --config 1m_1080p --worlds 1,2,4,8 > $O/band_sim_1m.jsonl 2> $O/band_sim_1m.err && \
timeout -k 10 400 python scripts/band_sim.py --config 5m_1080p --worlds 1,2,4,8 > $O/band_sim_5m.jsonl 2> $O/band_sim_5m.err && \
timeout -k 10 200 python bench.py --mode views --config 1k_256 --steps 100 --warmup 10 > $O/views_1k.json 2> $O/views_1k.err && \
timeout -k 10 200 python bench.py --mode views --config 100k_800 --steps 20 --warmup 3 > $O/views_100k.json 2> $O/views_100k.err && \
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py tests/test_gpu_shard_cpp.py tests/test_gpu_dist.py > $O/shard_tests.log 2>&1

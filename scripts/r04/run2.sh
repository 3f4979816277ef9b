#!/bin/bash
# round 4, GPU call 2: the configs[4] test, multi-GPU rehearsal at HEAD (one-launch pack, B2 band
# sum), the pack A/B at the 1M / 5M N = 8 shapes, and the F6-layout B1 variant A/B + parity
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
timeout -k 10 300 bash scripts/ab.sh $O/ab_lay.jsonl 3 b1lay && \
{ GSR_HIP_LIB=$R/3d_gaussian_splatting_amd/lib/variants/b1lay/libgsr_hip.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "golden or synthetic_parity or headline or checkpoint" > $O/parity_b1lay.log 2>&1; r=$?; [ $r -le 1 ]; }

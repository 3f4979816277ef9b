#!/bin/bash
# round 4, GPU call 19: the shipped merge build (merge marked unlikely) -- parity; four-wave F6 on
# every launch with 256-record (w4) or 128-record (w4b128) batches, in the post-reset loop and the
# 1M / 5M benches; b128 (band launches only) on the 1M N = 8 rehearsal
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_19
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXE=$R/3d_gaussian_splatting_amd/lib/gsr_train_loop
for v in base w4b128; do
  if [ $v = base ]; then L=""; else L=$R/3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so; fi
  { GSR_HIP_LIB=$L timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_views.py tests/test_gpu_train.py -k "golden or synthetic_parity or headline or deterministic or views or shard_path_equals or band_render or full_size or checkpoint or dense_tiles" > $O/parity_$v.log 2>&1; r=$?; [ $r -le 1 ]; } || exit 1
done
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m_reset.bin --gt 8000000 --init 6000000 --views 48 --iters 1200 --progress 100 --reset-interval 200 --densify-until 250 > $O/probe_write.log 2>&1 || exit 1
for v in base w4 w4b128 base w4b128; do
  if [ $v = base ]; then LP=""; else LP=$R/3d_gaussian_splatting_amd/lib/variants/$v; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 150 $EXE /tmp/loop6m_reset.bin $O/loop_$v.json > $O/loop_$v.log 2>&1 || { rc=$?; rm -f /tmp/loop6m_reset.bin; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['iters_per_s'], d['final_points'], d['binning_overflows'])" $O/loop_$v.json $v >> $O/loop_ab.txt
done
rm -f /tmp/loop6m_reset.bin
timeout -k 10 400 bash scripts/ab.sh $O/ab_1m.jsonl 2 nomerge w4 w4b128 || exit 1
AB_CONFIG=5m_1080p timeout -k 10 300 bash scripts/ab.sh $O/ab_5m.jsonl 1 w4b128 || exit 1
timeout -k 10 300 bash scripts/band_ab.sh $O/band_ab_1m.jsonl 2 1m_1080p 8 b128

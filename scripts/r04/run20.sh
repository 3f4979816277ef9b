#!/bin/bash
# round 4, GPU call 20: chunk merge at the batch end (bend: outside the blend loop) against the
# group-boundary merge (in-tree) and no merging -- parity, 1M A/B, post-reset loop
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_20
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXE=$R/3d_gaussian_splatting_amd/lib/gsr_train_loop
{ GSR_HIP_LIB=$R/3d_gaussian_splatting_amd/lib/variants/bend/libgsr_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_views.py tests/test_gpu_train.py -k "golden or synthetic_parity or headline or deterministic or views or shard_path_equals or band_render or full_size or checkpoint or dense_tiles" > $O/parity_bend.log 2>&1; r=$?; [ $r -le 1 ]; } || exit 1
timeout -k 10 500 bash scripts/ab.sh $O/ab_1m.jsonl 3 nomerge bend || exit 1
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m_reset.bin --gt 8000000 --init 6000000 --views 48 --iters 1200 --progress 100 --reset-interval 200 --densify-until 250 > $O/probe_write.log 2>&1 || exit 1
for v in base bend base bend; do
  if [ $v = base ]; then LP=""; else LP=$R/3d_gaussian_splatting_amd/lib/variants/$v; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 150 $EXE /tmp/loop6m_reset.bin $O/loop_$v.json > $O/loop_$v.log 2>&1 || { rc=$?; rm -f /tmp/loop6m_reset.bin; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['iters_per_s'], d['final_points'], d['binning_overflows'])" $O/loop_$v.json $v >> $O/loop_ab.txt
done
rm -f /tmp/loop6m_reset.bin

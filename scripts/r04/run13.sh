#!/bin/bash
# round 4, GPU call 13: the pre-sort gather writing raw rank-order rows that B2 converts
# (variant rankg; rankg_all also pre-sorts at 1M): parity, 1M / 5M bench A/B, loop A/B
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_13
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXE=$R/3d_gaussian_splatting_amd/lib/gsr_train_loop
for v in rankg rankg_all; do
  { GSR_HIP_LIB=$R/3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_views.py tests/test_gpu_train.py -k "golden or synthetic_parity or headline or deterministic or views or shard_path_equals or band_render or full_size" > $O/parity_$v.log 2>&1; r=$?; [ $r -le 1 ]; } || exit 1
done
timeout -k 10 300 bash scripts/ab.sh $O/ab_1m.jsonl 2 rankg_all || exit 1
AB_CONFIG=5m_1080p timeout -k 10 300 bash scripts/ab.sh $O/ab_5m.jsonl 2 rankg || exit 1
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m.bin --gt 8000000 --init 6000000 --views 48 --iters 4000 --progress 1000 > $O/probe_write.log 2>&1 || exit 1
for v in base rankg; do
  if [ $v = base ]; then LP=""; else LP=$R/3d_gaussian_splatting_amd/lib/variants/$v; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 150 $EXE /tmp/loop6m.bin $O/loop_$v.json > $O/loop_$v.log 2>&1 || { rc=$?; rm -f /tmp/loop6m.bin; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['iters_per_s'], d['final_points'], d['binning_overflows'])" $O/loop_$v.json $v >> $O/loop_ab.txt
done
rm -f /tmp/loop6m.bin

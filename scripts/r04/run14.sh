#!/bin/bash
# round 4, GPU call 14: the configs[4] loop's post-reset regime -- 6M Gaussians at 1280x832, one
# opacity reset at iteration 200, 1200 iterations (1000 after it) -- under a kernel trace; before
# it, the per-tile list / termination / chunk distribution around a reset; then the F6 variants
# (f6sync: termination from the batch barrier; f6pf: + software-pipelined batch loads) in that
# loop, their parity and the 1M bench A/B; b1w16: B1 batch windows of 1024 mask bytes
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_14
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXE=$R/3d_gaussian_splatting_amd/lib/gsr_train_loop
timeout -k 10 300 python -u scripts/deep_list_stats.py > $O/deep_list_stats.jsonl 2> $O/deep_list_stats.err
rc=$?; [ $rc -le 1 ] || exit $rc   # a Python error (1) still lets the trace run; a fault / time limit ends the call
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m_reset.bin --gt 8000000 --init 6000000 --views 48 --iters 1200 --progress 100 --reset-interval 200 --densify-until 250 > $O/probe_write.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/loop_trace -o t --output-format csv -- $EXE /tmp/loop6m_reset.bin $O/loop_reset.json > $O/loop_trace.log 2>&1) || { rc=$?; rm -f /tmp/loop6m_reset.bin; exit $rc; }
for v in base f6sync f6pf b1w16 f6pfw16 base; do
  if [ $v = base ]; then LP=""; else LP=$R/3d_gaussian_splatting_amd/lib/variants/$v; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 150 $EXE /tmp/loop6m_reset.bin $O/loop_$v.json > $O/loop_$v.log 2>&1 || { rc=$?; rm -f /tmp/loop6m_reset.bin; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['iters_per_s'], d['final_points'], d['binning_overflows'])" $O/loop_$v.json $v >> $O/loop_ab.txt
done
rm -f /tmp/loop6m_reset.bin
for v in f6pfw16 f6sync; do
  { GSR_HIP_LIB=$R/3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_views.py tests/test_gpu_train.py -k "golden or synthetic_parity or headline or deterministic or views or shard_path_equals or band_render or full_size" > $O/parity_$v.log 2>&1; r=$?; [ $r -le 1 ]; } || exit 1
done
timeout -k 10 300 bash scripts/ab.sh $O/ab_1m.jsonl 2 f6sync f6pf b1w16

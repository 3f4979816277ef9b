#!/bin/bash
# round 4, GPU call 6: splat-pack A/B at the 1M N = 8 shape, the 5M rehearsal, and library
# variants inside the configs[4] loop (6M Gaussians, 1280x832, 4000 iterations: past the first
# opacity reset) -- the executable picks up lib/variants/<name>/libgsr_hip.so through
# LD_LIBRARY_PATH (its RUNPATH comes after it) -- plus that loop's kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_6
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXE=$R/3d_gaussian_splatting_amd/lib/gsr_train_loop
timeout -k 10 600 bash scripts/band_ab.sh $O/band_ab_1m.jsonl 2 1m_1080p 8 packold pack1 pack2 || exit 1
timeout -k 10 400 python scripts/band_sim.py --config 5m_1080p --worlds 1,8 > $O/band_sim_5m.jsonl 2> $O/band_sim_5m.err || exit 1
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m.bin --gt 8000000 --init 6000000 --views 48 --iters 4000 --progress 1000 > $O/probe_write.log 2>&1 || exit 1
for v in base nopresort adam2 adamnt adam2nt; do
  if [ $v = base ]; then LP=""; else LP=$R/3d_gaussian_splatting_amd/lib/variants/$v; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 150 $EXE /tmp/loop6m.bin $O/loop_$v.json > $O/loop_$v.log 2>&1 || { rc=$?; rm -f /tmp/loop6m.bin; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['iters_per_s'], d['final_points'], d['binning_overflows'])" $O/loop_$v.json $v >> $O/loop_ab.txt
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/loop_trace -o t --output-format csv -- $EXE /tmp/loop6m.bin $O/loop4k.json > $O/loop_trace.log 2>&1)
rc=$?
rm -f /tmp/loop6m.bin
exit $rc

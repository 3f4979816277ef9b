#!/bin/bash
# round 4, GPU call 10: stripe masks in the sort values -- the GPU suite minus configs[4], the
# 1M / 5M bench A/B against the previous library (bytemask), and the configs[4] loop A/B
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_10
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXE=$R/3d_gaussian_splatting_amd/lib/gsr_train_loop
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "not configs4" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 bash scripts/ab.sh $O/ab_1m.jsonl 3 bytemask || exit 1
AB_CONFIG=5m_1080p timeout -k 10 300 bash scripts/ab.sh $O/ab_5m.jsonl 2 bytemask || exit 1
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m.bin --gt 8000000 --init 6000000 --views 48 --iters 4000 --progress 1000 > $O/probe_write.log 2>&1 || exit 1
for v in base bytemask; do
  if [ $v = base ]; then LP=""; else LP=$R/3d_gaussian_splatting_amd/lib/variants/$v; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 150 $EXE /tmp/loop6m.bin $O/loop_$v.json > $O/loop_$v.log 2>&1 || { rc=$?; rm -f /tmp/loop6m.bin; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['iters_per_s'], d['final_points'], d['binning_overflows'])" $O/loop_$v.json $v >> $O/loop_ab.txt
done
rm -f /tmp/loop6m.bin

#!/bin/bash
# round 4, GPU call 5: A/B of library variants inside the configs[4] loop (6M Gaussians,
# 1280x832, 2000 iterations): the executable picks up lib/variants/<name>/libgsr_hip.so through
# LD_LIBRARY_PATH (its RUNPATH comes after it)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_5
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXE=$R/3d_gaussian_splatting_amd/lib/gsr_train_loop
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m.bin --gt 8000000 --init 6000000 --views 48 --iters 2000 --progress 500 > $O/probe_write.log 2>&1 || exit 1
for r in 1 2; do
  for v in base nopresort adam2 adamnt adam2nt b1lay; do
    if [ $v = base ]; then LP=""; else LP=$R/3d_gaussian_splatting_amd/lib/variants/$v; fi
    LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 $EXE /tmp/loop6m.bin $O/loop_${v}_$r.json > $O/loop_${v}_$r.log 2>&1 || { rc=$?; rm -f /tmp/loop6m.bin; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['iters_per_s'], d['final_points'], d['binning_overflows'])" $O/loop_${v}_$r.json $v >> $O/loop_ab.txt
  done
done
rm -f /tmp/loop6m.bin

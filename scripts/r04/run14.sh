#!/bin/bash
# round 4, GPU call 14: the configs[4] loop's post-reset regime under a kernel trace -- 6M
# Gaussians at 1280x832, one opacity reset at iteration 200, 1200 iterations (1000 after it);
# before it, the per-tile list / termination / chunk distribution around a reset
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
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/loop_trace -o t --output-format csv -- $EXE /tmp/loop6m_reset.bin $O/loop_reset.json > $O/loop_trace.log 2>&1)
rc=$?
rm -f /tmp/loop6m_reset.bin
exit $rc

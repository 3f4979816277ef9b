#!/bin/bash
# round 4, GPU call 3: presort threshold checks (2.5M oracle case, views past it), the single-GPU
# variant A/B at 1M and 5M with their parity, and the configs[4] loop's kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_3
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_views.py \
  -k "headline or presort_switch or full_size" > $O/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 bash scripts/ab.sh $O/ab_1m.jsonl 2 b1pf b1cmp f1persist b2persist f1b2persist presort1m && \
AB_CONFIG=5m_1080p timeout -k 10 400 bash scripts/ab.sh $O/ab_5m.jsonl 2 nopresort f1b2persist && \
for v in f1b2persist b1cmp b1pf; do
  { GSR_HIP_LIB=$R/3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "golden or synthetic_parity or headline" > $O/parity_$v.log 2>&1; r=$?; [ $r -le 1 ]; } || exit 9
done && \
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m.bin --gt 8000000 --init 6000000 --views 48 --iters 2000 --progress 250 > $O/probe_write.log 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/loop_trace -o t --output-format csv -- $R/3d_gaussian_splatting_amd/lib/gsr_train_loop /tmp/loop6m.bin $O/loop2k.json > $O/loop_trace.log 2>&1)
rc=$?
rm -f /tmp/loop6m.bin
exit $rc

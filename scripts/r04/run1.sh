#!/bin/bash
# round 4, GPU call 1: DMA-offset fix parity, baseline bench, configs[4] loop probe at ~6M
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "allocation_end or golden or synthetic_parity or deterministic or checkpoint or headline" > $O/tests.log 2>&1 && \
{ timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_views.py tests/test_gpu_batch.py > $O/tests_views.log 2>&1; r=$?; [ $r -le 1 ]; } && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_shard_cpp.py tests/test_gpu_train.py tests/test_gpu_dropin.py tests/test_gpu_train_loop.py -k "not configs4" > $O/tests_train.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 python bench.py --mode views --config 1k_256 --steps 100 --warmup 10 > $O/views_1k.json 2> $O/views_1k.err && \
timeout -k 10 200 python bench.py --mode views --config 100k_800 --steps 20 --warmup 3 > $O/views_100k.json 2> $O/views_100k.err && \
timeout -k 10 600 bash scripts/ab.sh $O/ab_b1.jsonl 2 b1pf b1cmp f1persist b2persist f1b2persist && \
AB_CONFIG=5m_1080p timeout -k 10 400 bash scripts/ab.sh $O/ab_5m.jsonl 2 nopresort f1b2persist && \
for v in f1b2persist b1cmp b1pf; do
  { GSR_HIP_LIB=$R/3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "golden or synthetic_parity or headline" > $O/parity_$v.log 2>&1; r=$?; [ $r -le 1 ]; } || exit 9
done && \
timeout -k 10 300 python scripts/loop_probe.py /tmp/loop6m.bin --gt 8000000 --init 6000000 --views 48 --iters 2000 --progress 250 > $O/probe_write.log 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/loop_trace -o t --output-format csv -- $R/3d_gaussian_splatting_amd/lib/gsr_train_loop /tmp/loop6m.bin $O/loop2k.json > $O/loop_trace.log 2>&1) && \
rm -f /tmp/loop6m.bin
rc=$?
rm -f /tmp/loop6m.bin
exit $rc

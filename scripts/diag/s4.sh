set -o pipefail
O=gpurun_out/s4
mkdir -p $O
R=$GRAFT_REPO_ROOT
V=$R/3d_gaussian_splatting_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for c in 1m_1080p 5m_1080p; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit $?
for v in lsd depth; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --lib $V/$v/libgsr_hip.so > $O/bench_${c}_$v.json 2>> $O/bench.err || exit $?
done
done
GSR_HIP_LIB=$V/depth/libgsr_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > $O/tests_depth.log 2>&1
echo "depth tests rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t5 -o t --output-format csv -- python3 $R/bench.py --config 5m_1080p --steps 10 --warmup 3 --no-cpu-baseline --no-stage-events > $R/$O/t5.json 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t5d -o t --output-format csv -- python3 $R/bench.py --config 5m_1080p --steps 10 --warmup 3 --no-cpu-baseline --no-stage-events --lib $V/depth/libgsr_hip.so > $R/$O/t5d.json 2>&1 || exit $?

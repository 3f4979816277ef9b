set -o pipefail
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
for c in 1m_1080p 5m_1080p; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit $?
for v in gidorder lsd; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --lib 3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so > $O/bench_${c}_$v.json 2>> $O/bench.err || exit $?
done
done

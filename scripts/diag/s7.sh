set -o pipefail
O=gpurun_out/s7
mkdir -p $O
V=3d_gaussian_splatting_amd/lib/variants
for rep in 1 2; do
timeout -k 10 150 python bench.py --config 5m_1080p --no-cpu-baseline > $O/b_base_$rep.json 2>> $O/bench.err || exit $?
for v in ts8k512 ts8k1024; do
timeout -k 10 150 python bench.py --config 5m_1080p --no-cpu-baseline --lib $V/$v/libgsr_hip.so > $O/b_${v}_$rep.json 2>> $O/bench.err || exit $?
done
done
GSR_HIP_LIB=$PWD/$V/ts8k512/libgsr_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "dense or 5m or deep" > $O/tests.log 2>&1
echo "tests rc=$?"

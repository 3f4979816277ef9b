set -o pipefail
O=gpurun_out/s13
mkdir -p $O
V=3d_gaussian_splatting_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
for c in 1m_1080p 5m_1080p; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_base_$rep.json 2>> $O/err || exit $?
for v in nomsd msd32 msd128; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --lib $V/$v/libgsr_hip.so > $O/b_${c}_${v}_$rep.json 2>> $O/err || exit $?
done
done
done

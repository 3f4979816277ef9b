set -o pipefail
O=gpurun_out/s5
mkdir -p $O
R=$GRAFT_REPO_ROOT
V=$R/3d_gaussian_splatting_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "synthetic or headline or dense or capacity or golden" > $O/tests.log 2>&1 || exit $?
for c in 1m_1080p 5m_1080p; do
for rep in 1 2; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/bench_${c}_$rep.json 2>> $O/bench.err || exit $?
for v in noxcd radixonly; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --lib $V/$v/libgsr_hip.so > $O/bench_${c}_${v}_$rep.json 2>> $O/bench.err || exit $?
done
done
done

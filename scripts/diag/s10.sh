set -o pipefail
O=gpurun_out/s10
mkdir -p $O
V=3d_gaussian_splatting_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_init.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
timeout -k 10 300 python scripts/band_sim.py --config 1m_1080p --worlds 8 --no-single > $O/band_1m_base_$rep.jsonl 2>> $O/err || exit $?
timeout -k 10 300 python scripts/band_sim.py --config 1m_1080p --worlds 8 --no-single --lib $V/bigtile/libgsr_hip.so > $O/band_1m_bigtile_$rep.jsonl 2>> $O/err || exit $?
timeout -k 10 150 python bench.py --config 100k_800 --no-cpu-baseline > $O/b100k_base_$rep.json 2>> $O/err || exit $?
timeout -k 10 150 python bench.py --config 100k_800 --no-cpu-baseline --lib $V/bigtile/libgsr_hip.so > $O/b100k_bigtile_$rep.json 2>> $O/err || exit $?
done

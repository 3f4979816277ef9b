set -o pipefail
O=gpurun_out/s8
mkdir -p $O
V=3d_gaussian_splatting_amd/lib/variants
for c in 1m_1080p 5m_1080p; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_base.json 2>> $O/bench.err || exit $?
for v in gdiag1 gdiag2; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --lib $V/$v/libgsr_hip.so > $O/b_${c}_$v.json 2>> $O/bench.err || exit $?
done
done

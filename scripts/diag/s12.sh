set -o pipefail
O=gpurun_out/s12
mkdir -p $O
V=3d_gaussian_splatting_amd/lib/variants
for rep in 1 2; do
for c in 1m_1080p 5m_1080p; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_base_$rep.json 2>> $O/err || exit $?
for v in ri8 ri12 ri24; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --lib $V/$v/libgsr_hip.so > $O/b_${c}_${v}_$rep.json 2>> $O/err || exit $?
done
done
done

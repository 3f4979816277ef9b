set -o pipefail
O=gpurun_out/s14
mkdir -p $O
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 python bench.py --config 5m_1080p --no-cpu-baseline > $O/bench_5m.json 2>> $O/bench.err || exit $?
timeout -k 10 200 python bench.py --mode train --no-cpu-baseline > $O/bench_train.json 2>> $O/bench.err || exit $?
V=3d_gaussian_splatting_amd/lib/variants
for rep in 1 2; do
for c in 1m_1080p 5m_1080p; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_base_$rep.json 2>> $O/err || exit $?
for v in ri8 ri12; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --lib $V/$v/libgsr_hip.so > $O/b_${c}_${v}_$rep.json 2>> $O/err || exit $?
done
done
done

set -o pipefail
O=gpurun_out/s3
mkdir -p $O
R=$GRAFT_REPO_ROOT
V=$R/3d_gaussian_splatting_amd/lib/variants
GSR_HIP_LIB=$V/cnt/libgsr_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "synthetic or headline or dense or capacity or band or shard" > $O/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for c in 1m_1080p 5m_1080p; do
for v in cnt cntgid; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t_${c}_$v -o t --output-format csv -- python3 $R/bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-stage-events --lib $V/$v/libgsr_hip.so > $R/$O/t_${c}_$v.json 2>&1 || exit $?
done
done

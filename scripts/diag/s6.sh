set -o pipefail
O=gpurun_out/s6
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "synthetic or headline or dense or capacity or golden" > $O/tests.log 2>&1 || exit $?
for c in 1m_1080p 5m_1080p; do
timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/bench_${c}.json 2>> $O/bench.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t1 -o t --output-format csv -- python3 $R/bench.py --config 1m_1080p --steps 10 --warmup 3 --no-cpu-baseline --no-stage-events > $R/$O/t1.json 2>&1 || exit $?

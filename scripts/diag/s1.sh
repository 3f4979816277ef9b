set -o pipefail
O=gpurun_out/s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 python bench.py --config 5m_1080p --no-cpu-baseline > $O/bench_5m.json 2>> $O/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/t5m -o t5m --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 5m_1080p --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/t5m.log 2>&1

set -o pipefail
O=gpurun_out/${1:-r01z}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 python bench.py --config 5m_1080p --no-cpu-baseline > $O/bench_5m.json 2>> $O/bench.err && \
timeout -k 10 200 python bench.py --mode train --no-cpu-baseline > $O/bench_train.json 2>> $O/bench.err && \
timeout -k 10 900 bash scripts/profile_round.sh ${1:-r01z}_prof > $O/prof.log 2>&1

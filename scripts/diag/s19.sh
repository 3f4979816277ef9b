set -o pipefail
O=gpurun_out/s19
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config 5m_1080p --no-cpu-baseline > $O/bench_5m.json 2>> $O/bench.err || exit $?
timeout -k 10 900 bash scripts/profile_round.sh r03c_prof > $O/prof.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > $O/bench.json 2>> $O/bench.err || exit $?

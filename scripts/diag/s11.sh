set -o pipefail
O=gpurun_out/s11
mkdir -p $O
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 python bench.py --config 5m_1080p --no-cpu-baseline > $O/bench_5m.json 2>> $O/bench.err || exit $?
timeout -k 10 900 bash scripts/profile_round.sh r03b_prof > $O/prof.log 2>&1

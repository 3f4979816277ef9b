set -o pipefail
O=gpurun_out/s15
mkdir -p $O
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench2.json 2>> $O/bench.err || exit $?
timeout -k 10 200 python bench.py --config 5m_1080p --no-cpu-baseline > $O/bench_5m.json 2>> $O/bench.err || exit $?

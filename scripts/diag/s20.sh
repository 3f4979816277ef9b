set -o pipefail
O=gpurun_out/s20
mkdir -p $O
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?

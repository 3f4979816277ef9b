set -o pipefail
O=gpurun_out/s18
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/t5 -o t --output-format csv -- python3 $R/bench.py --config 5m_1080p --steps 10 --warmup 3 --no-cpu-baseline --no-stage-events > $R/$O/t5.json 2>&1 || exit $?

#!/bin/bash
# round 4, GPU call 15: the end-of-round profile of the shipped library (kernel trace + PMC
# passes, scripts/profile_round.sh), the bench line, the 5M / train benches and smoke()
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_15
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 bash scripts/profile_round.sh r04_prof2 > $O/profile.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_head.json 2> $O/bench_head.err || exit 1
timeout -k 10 200 python bench.py --config 5m_1080p --no-cpu-baseline > $O/bench_5m.json 2> $O/bench_5m.err || exit 1
timeout -k 10 200 python bench.py --mode train --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1

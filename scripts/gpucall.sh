#!/bin/bash
# One parametrised GPU call (run on the box by gpurun):  scripts/gpucall.sh TAG STEP [STEP ...]
# Every step runs under its own time limit, writes gpurun_out/TAG/NN_<name>.log, and the call
# stops at the first step that ends like a GPU fault, abort, segfault or time limit (never
# starting another GPU step after one); plain test failures (rc 1) go on to the next step.
# Steps:
#   suite                      the whole `pytest -m gpu` suite as the driver runs it
#   tests:ARGS                 pytest -m gpu ARGS (files, -k EXPR ...; ':' inside ARGS is kept)
#   smoke                      __graft_entry__.smoke()
#   bench:ARGS                 python bench.py ARGS  (the JSON line goes to NN_bench.json too)
#   bandsim:CONFIG:WORLDS      scripts/band_sim.py --config CONFIG --worlds WORLDS
#   prof:NAME                  scripts/profile_round.sh NAME (kernel trace + PMC passes)
#   ab:OUT:ROUNDS:VARIANTS     scripts/ab.sh OUT ROUNDS VARIANTS (space-separated by ',')
#   cmd:SECONDS:COMMAND        any other command, with its own limit
# The calls of each round and what they produced are listed in scripts/gpucalls.md.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  case $kind in
    suite)   name=suite;   lim=1100; cmd="python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu tests" ;;
    tests)   name=tests;   lim=900;  cmd="$PYT $arg" ;;
    smoke)   name=smoke;   lim=300;  cmd="python -u -c 'import __graft_entry__ as g; g.smoke()'" ;;
    bench)   name=bench;   lim=600;  cmd="python -u bench.py $arg" ;;
    bandsim) name=bandsim; lim=600;  cmd="python -u scripts/band_sim.py --config ${arg%%:*} --worlds ${arg#*:}" ;;
    prof)    name=prof;    lim=900;  cmd="bash scripts/profile_round.sh $arg" ;;
    ab)      name=ab;      lim=900;  IFS=: read -r o rr vv <<< "$arg"; cmd="bash scripts/ab.sh $o $rr ${vv//,/ }" ;;
    cmd)     name=cmd;     lim=${arg%%:*}; cmd=${arg#*:} ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  log=$(printf "%s/%02d_%s.log" "$O" $n $name)
  echo "=== [$TAG $n] $cmd  (limit ${lim}s) -> $log"
  timeout -k 10 "$lim" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  echo "=== [$TAG $n] rc=$rc"
  tail -3 "$log"
  if [ $name = bench ]; then grep '^{' "$log" | tail -1 > "${log%.log}.json"; fi
  case $rc in
    0|1|2|4|5) ;;
    *) echo "=== stopping after rc=$rc (no further GPU step in this call)"; exit $rc ;;
  esac
done

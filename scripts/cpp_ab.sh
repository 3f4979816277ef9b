#!/bin/bash
# A/B of experimental library builds on the whole-C++-step rehearsal (scripts/band_sim.py --cpp):
# the in-tree library and each variant (lib/variants/<name>) interleaved, ROUNDS times; one line
# per run with the slowest rank's compute-only and with-copies step times.
# usage: scripts/cpp_ab.sh OUTFILE ROUNDS CONFIG WORLD name1 [name2 ...]
set -u
OUT=$1; ROUNDS=$2; CFG=$3; WORLD=$4; shift 4
run() {  # $1 = variant label, rest = extra args
  local v=$1; shift
  timeout -k 10 300 python3 scripts/band_sim.py --config $CFG --worlds $WORLD --no-single --steps 7 --cpp "$@" 2>/dev/null \
    | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{') and 'compute' in l:
        d=json.loads(l); print(json.dumps({'variant':sys.argv[1],'world':d['world'],'compute_ms':d['compute']['slowest_rank_ms'],
              'with_copies_ms':d['with_copies']['slowest_rank_ms'],'rank_ms':d['compute']['rank_ms']}))" $v >> $OUT
}
for r in $(seq 1 $ROUNDS); do
  run base || exit $?
  for v in "$@"; do run $v --lib 3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so || exit $?; done
done

#!/bin/bash
# A/B of experimental library builds on the multi-GPU rehearsal: scripts/band_sim.py at one world
# size, the in-tree library and each variant (lib/variants/<name>) interleaved, ROUNDS times.
# usage: scripts/band_ab.sh OUTFILE ROUNDS CONFIG WORLD name1 [name2 ...]
set -u
OUT=$1; ROUNDS=$2; CFG=$3; WORLD=$4; shift 4
for r in $(seq 1 $ROUNDS); do
  timeout -k 10 200 python3 scripts/band_sim.py --config $CFG --worlds $WORLD --no-single --steps 5 2>/dev/null \
    | python3 -c "import json,sys; [print(json.dumps({'variant':'base', **json.loads(l)})) for l in sys.stdin if 'slowest_rank_ms' in l]" >> $OUT || exit $?
  for v in "$@"; do
    timeout -k 10 200 python3 scripts/band_sim.py --config $CFG --worlds $WORLD --no-single --steps 5 \
      --lib 3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so 2>/dev/null \
      | python3 -c "import json,sys; [print(json.dumps({'variant':sys.argv[1], **json.loads(l)})) for l in sys.stdin if 'slowest_rank_ms' in l]" $v >> $OUT || exit $?
  done
done

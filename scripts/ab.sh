#!/bin/bash
# A/B timing of experimental library builds (lib/variants/<name>/libgsr_hip.so from
# _build.build_variant) against the in-tree library: bench.py runs interleaved, ROUNDS times.
# usage: [AB_CONFIG=5m_1080p] scripts/ab.sh OUTFILE ROUNDS name1 [name2 ...]
set -u
OUT=$1; ROUNDS=$2; shift 2
CFG=${AB_CONFIG:-1m_1080p}
for r in $(seq 1 $ROUNDS); do
  timeout -k 10 150 python3 bench.py --config $CFG --no-cpu-baseline --steps 30 --warmup 5 > /tmp/ab_base.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('/tmp/ab_base.json')); print(json.dumps({'variant':'base','value':d['value'],'stage_ms':d.get('stage_ms')}))" >> $OUT
  for v in "$@"; do
    timeout -k 10 150 python3 bench.py --config $CFG --no-cpu-baseline --steps 30 --warmup 5 --lib 3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so > /tmp/ab_v.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open('/tmp/ab_v.json')); print(json.dumps({'variant':sys.argv[1],'value':d['value'],'stage_ms':d.get('stage_ms')}))" $v >> $OUT
  done
done

"""Summarise an ab.sh / cpp_ab.sh JSONL file: per variant, the values and the mean stage times."""
import collections
import json
import sys

for path in sys.argv[1:]:
    d = collections.defaultdict(list)
    for line in open(path):
        r = json.loads(line)
        d[r['variant']].append(r)
    print(path)
    for k, v in d.items():
        vals = [round(x['value'], 1) for x in v]
        st = v[0].get('stage_ms') or {}
        means = {s: round(sum((x.get('stage_ms') or {}).get(s, 0) for x in v) / len(v), 3) for s in st}
        print('  %-10s %s  mean %.1f  %s' % (k, vals, sum(x['value'] for x in v) / len(v), means))

set -o pipefail
timeout -k 10 300 python -u scripts/diag/binning_determinism.py > gpurun_out/r03_diag_binning.log 2>&1; echo diag_rc=$?
tail -12 gpurun_out/r03_diag_binning.log
for cfg in 1m_1080p 5m_1080p; do
  AB_CONFIG=$cfg timeout -k 10 900 bash scripts/ab.sh gpurun_out/r03_ab_sort_$cfg.jsonl 2 sort512 sort1024 || exit $?
done
cat gpurun_out/r03_ab_sort_*.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); s = d['stage_ms'] or {}
    print(d['variant'], d['value'], s.get('depth_sort'), s.get('tile_sort'))"

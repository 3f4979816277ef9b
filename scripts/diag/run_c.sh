set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_init.py tests/test_gpu_train_loop.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_c.log 2>&1; rc=$?; tail -5 gpurun_out/r03_gpu_c.log; case $rc in 0|1) ;; *) exit $rc;; esac
for cfg in 1m_1080p 5m_1080p; do
  AB_CONFIG=$cfg timeout -k 10 900 bash scripts/ab.sh gpurun_out/r03_ab_rank_$cfg.jsonl 2 rank_seq rank_slice_only || exit $?
done
cat gpurun_out/r03_ab_rank_*.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); s = d['stage_ms'] or {}
    print(d['variant'], d['value'], s.get('depth_sort'), s.get('tile_sort'))"

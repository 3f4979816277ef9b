set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_autograd.py tests/test_gpu_train.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_e.log 2>&1; rc=$?; tail -5 gpurun_out/r03_gpu_e.log; case $rc in 0|1) ;; *) exit $rc;; esac
for cfg in 1m_1080p 5m_1080p; do
  AB_CONFIG=$cfg timeout -k 10 900 bash scripts/ab.sh gpurun_out/r03_ab_e_$cfg.jsonl 2 granule0 granule8 f1_chunks || exit $?
done
cat gpurun_out/r03_ab_e_*.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); s = d['stage_ms'] or {}
    print(d['variant'], d['value'], 'F1', s.get('preprocess'), 'F6', s.get('blend_fwd'), 'B1', s.get('blend_bwd'))"

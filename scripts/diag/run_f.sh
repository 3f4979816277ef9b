set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_f.log 2>&1; rc=$?; tail -5 gpurun_out/r03_gpu_f.log; case $rc in 0|1) ;; *) exit $rc;; esac
for cfg in 1m_1080p 5m_1080p; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r03_bench_f_$cfg.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['stage_ms'])" gpurun_out/r03_bench_f_$cfg.json
done
LOOP_ITERS=30000 bash scripts/diag/run_loop.sh

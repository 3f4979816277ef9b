set -o pipefail
O=gpurun_out/s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/band_sim.py --config 1m_1080p > $O/band_1m.jsonl 2> $O/band.err || exit $?
timeout -k 10 300 python scripts/band_sim.py --config 5m_1080p > $O/band_5m.jsonl 2>> $O/band.err || exit $?

set -o pipefail
O=gpurun_out/s17
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?

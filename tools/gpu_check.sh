# GPU-box check: kernel parity tests then smoke(); stops at the first crash-like exit.
set -u
TAG=${1:-run}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/$TAG-tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/$TAG-tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG-smoke.log 2>&1
echo "smoke rc=$?" >> gpurun_out/$TAG-smoke.log

# GPU-box, round 3: the whole -m gpu suite, smoke(), the band probe, the default bench line and a
# kernel-stats pass of the short bench, each step under its own limit; the first failure ends it.
#   bash tools/gpu_r03.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r03}
O=gpurun_out/$T
mkdir -p $O
export AZ_REPORT_DIR=$O/reports
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --durations=30 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/band_probe.py 512 20 > $O/band_probe.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 200 --warmup 200 --no-cpu --no-selfplay --no-train --no-agg-extra --large-batch 0 > $O/kt.log 2>&1 || exit $?
echo done > $O/done

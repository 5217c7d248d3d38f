# GPU-box, round 6: the evidence at HEAD -- the whole GPU suite (margins reported),
# smoke(), the driver's bench command, and a kernel trace (--stats) of the B = 512 step.
#   bash tools/gpu_r06_final.sh TAG
set -u
TAG=${1:-r06final}
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/$TAG
mkdir -p $R
export AZ_REPORT_DIR=$R/reports
timeout -k 10 840 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > $R/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $R/bench.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o step -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-selfplay --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 > $R/kt.log 2>&1 || exit $?
echo done > $R/done
# the self-play leg's kernels (two lanes; durations include the lanes' overlap)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/sp -o sp -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0 > $R/sp.log 2>&1 || exit $?
echo done > $R/done_sp

# GPU-box: the round's evidence in one call -- GPU tests, the default bench line, and a
# rocprofv3 kernel trace of a short bench run.  Every step has its own time limit; the first
# failure ends the script.
#   bash tools/gpu_round.sh TAG
set -eu
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
export AZ_REPORT_DIR=$O/reports
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-selfplay --no-train --large-batch 0 > $O/kt.log 2>&1
echo done > $O/done

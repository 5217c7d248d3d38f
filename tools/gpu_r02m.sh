# GPU-box (r02m): gemm_x3 at small M (dispatch threshold), then the round evidence: GPU tests,
# bench line, kernel stats, FETCH/WRITE PMC passes of the bench step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r02m}
O=gpurun_out/$T
mkdir -p $O
AZ_TUNING_LIB=1 timeout -k 10 300 python tools/gemm_sweep.py x3 32,48,64,96,65536 2 auto > $O/x3_small.jsonl 2> $O/x3_small.err || exit $?
export AZ_REPORT_DIR=$O/reports
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-selfplay --no-train --no-agg-extra --large-batch 0 > $O/kt.log 2>&1 || exit $?
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --no-selfplay --no-train --no-agg-extra --no-grid --no-b1 --large-batch 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit $?
echo done > $O/done

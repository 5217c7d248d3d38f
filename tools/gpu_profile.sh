# GPU-box: GPU tests, the bench line, a rocprofv3 kernel-trace/stats pass and two PMC passes
# (FETCH_SIZE, WRITE_SIZE in separate runs, MI355X_MICROARCH.md §rocprofv3 PMC slots).
set -u
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
# kernel stats of the B = 512 step (+ aggregate / grid legs) alone, so the GEMM tile kernel's
# average is the bench's roofline kernel; then the train + large-batch legs in a pass of their own
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-selfplay --no-agg-extra --no-train --large-batch 0 > $OUT/stats.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_tl -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-selfplay --no-aggregate --no-grid > $OUT/stats_tl.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-selfplay --no-train --no-agg-extra --large-batch 0 > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-selfplay --no-train --no-agg-extra --large-batch 0 > $OUT/write.log 2>&1 || exit $?
echo done > $OUT/done

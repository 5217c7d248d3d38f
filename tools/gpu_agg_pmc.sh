# GPU-box: FETCH_SIZE / WRITE_SIZE (separate passes) of the aggregate leg incl. the cold-cache and
# 4096-grid launches; summarised by tools/agg_pmc_report.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/aggpmc
mkdir -p $O
Q="--no-cpu --no-selfplay --no-train --no-grid --large-batch 0 --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py $Q > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py $Q > $O/write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $Q > $O/kt.log 2>&1 || exit $?

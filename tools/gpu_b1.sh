# GPU-box: the batch-1 leaf chain -- the bench's as_called_b1 leg alone, then its kernel stats.
#   bash tools/gpu_b1.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-b1}
O=gpurun_out/$T
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --no-selfplay --no-train --no-aggregate --no-grid --large-batch 0"
timeout -k 10 300 $B > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit $?
echo done > $O/done

# GPU-box: round-4 evidence at HEAD (tools/gpu_r04.sh) then the HBM-byte passes of the bench's
# B = 512 legs (FETCH_SIZE / WRITE_SIZE, separate runs).   bash tools/gpu_r04x.sh TAG
set -u
T=${1:-r04x}
bash tools/gpu_r04.sh $T || exit 1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$T
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --settle-ms 0 --no-cpu --no-selfplay --no-train --no-agg-extra --no-grid --no-b1 --large-batch 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit $?
echo done > $OUT/done

# GPU-box: the FETCH_SIZE / WRITE_SIZE passes (separate runs) behind profiles/pmc.json: the bench's
# B = 512 step and the fused GNN layer probe (512 grids, source projection + 23 fused launches).
#   bash tools/gpu_pmc_r02.sh TAG
set -u
TAG=${1:-r02}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --no-selfplay --no-train --no-agg-extra --no-grid --no-b1 --large-batch 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ffetch -o run -- python3 tools/fused_probe.py one > $OUT/ffetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/fwrite -o run -- python3 tools/fused_probe.py one > $OUT/fwrite.log 2>&1 || exit $?
echo done > $OUT/done

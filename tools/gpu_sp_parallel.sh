# GPU-box: self-play games/s against the games in flight (bench.py --sp-parallel), alternating.
#   bash tools/gpu_sp_parallel.sh TAG "P list"
set -u
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/${1:-spp}; mkdir -p $R
for i in 1 2; do
  for p in ${2:-0 6144 4096 2048}; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0 --sp-parallel $p > $R/sp_p${p}_$i.json 2>> $R/err.txt || exit $?
  done
done

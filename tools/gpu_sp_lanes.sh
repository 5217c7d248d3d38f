# GPU-box: self-play games/s against the number of lanes (bench.py --sp-lanes), alternating.
#   bash tools/gpu_sp_lanes.sh TAG "L list"
set -u
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/${1:-lanes}; mkdir -p $R
for i in 1 2; do
  for l in ${2:-2 3}; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0 --sp-lanes $l > $R/sp_l${l}_$i.json 2>> $R/err.txt || exit $?
  done
done

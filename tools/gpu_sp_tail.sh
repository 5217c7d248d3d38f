# GPU-box: self-play games/s with the lane's engine threads cut once few games are left
# (AZ_SP_TAIL_SLOTS_PER_THREAD: 16 default, 0 = always all threads), alternating.
#   bash tools/gpu_sp_tail.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/${1:-tail}; mkdir -p $R
for i in 1 2 3; do
  for t in 16 0; do
    AZ_SP_TAIL_SLOTS_PER_THREAD=$t timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0 > $R/sp_t${t}_$i.json 2>> $R/err.txt || exit $?
  done
done

set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/nbs; mkdir -p $O
B="python bench.py --steps 200 --warmup 20 --no-cpu --no-selfplay --no-grid --no-train --no-b1 --no-aggregate --large-batch 0"
for r in 1 2; do
  AZ_TUNING_LIB=1 timeout -k 10 200 $B > $O/model_$r.log 2>&1 || exit 1
  for nb in 1 2 3 4; do AZ_TUNING_LIB=1 AZ_TRUNK_NB=$nb timeout -k 10 200 $B > $O/nb${nb}_$r.log 2>&1 || exit 1; done
done
echo done > $O/done

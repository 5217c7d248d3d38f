# Self-play leg with the heads variants (tuning build for every run): one-launch R = 4 (product),
# R = 8, two-pass.   bash tools/gpu_ab_spheads.sh <tag>
set -e
tag=${1:-ab_spheads}
mkdir -p gpurun_out/$tag
export AZ_TUNING_LIB=1
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2; do
  for mode in default r8 twopass; do
    unset AZ_HEADS_R AZ_HEADS_TWOPASS
    if [ $mode = r8 ]; then export AZ_HEADS_R=8; fi
    if [ $mode = twopass ]; then export AZ_HEADS_TWOPASS=1; fi
    timeout -k 10 200 python -u bench.py $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['selfplay']; print(json.dumps({'mode':'$mode','games_per_s':s['games_per_s'],'net_wait_s':s['net_wait_s'],'host_s':s['host_s']}))" >> gpurun_out/$tag/ab.jsonl
  done
done

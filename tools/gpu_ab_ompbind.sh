# A/B of the self-play leg with and without the engine's OpenMP binding, alternated, one session
#   bash tools/gpu_ab_ompbind.sh <tag>
set -e
tag=${1:-ab_omp}
mkdir -p gpurun_out/$tag
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2; do
  for mode in nobind bind; do
    if [ $mode = nobind ]; then export AZ_OMP_NO_BIND=1; else unset AZ_OMP_NO_BIND; fi
    timeout -k 10 200 python -u bench.py $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['selfplay']; print(json.dumps({'mode':'$mode','games_per_s':s['games_per_s'],'net_wait_s':s['net_wait_s'],'host_s':s['host_s'],'host_only_gps':s.get('host_only',{}).get('games_per_s')}))" >> gpurun_out/$tag/ab.jsonl
  done
done

# Self-play leg vs engine thread count and OpenMP wait policy (the rank's cgroup quota is 16 CPUs
# and the main thread, the HIP runtime and idle-spinning OpenMP workers share it), alternated in
# one GPU session.   bash tools/gpu_ab_spthreads.sh <tag>
set -e
tag=${1:-ab_spthreads}
mkdir -p gpurun_out/$tag
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2; do
  for mode in 16 15 14 12 16p 15p; do
    th=${mode%p}
    if [ "$mode" != "$th" ]; then export OMP_WAIT_POLICY=passive; else unset OMP_WAIT_POLICY; fi
    timeout -k 10 200 python -u bench.py $F --sp-threads $th 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['selfplay']; print(json.dumps({'mode':'$mode','games_per_s':s['games_per_s'],'net_wait_s':s['net_wait_s'],'host_s':s['host_s'],'assemble_s':s.get('assemble_s')}))" >> gpurun_out/$tag/ab.jsonl
  done
done

# Self-play leg: lanes on their own streams vs one stream (AZ_SP_ONE_STREAM=1), 2 / 3 lanes,
# OpenMP passive wait, one GPU session.   bash tools/gpu_ab_spstream.sh <tag>
set -e
tag=${1:-ab_spstream}
mkdir -p gpurun_out/$tag
export OMP_WAIT_POLICY=passive
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2; do
  for mode in own:2 one:2 own:3 one:3 one:4; do
    st=${mode%%:*}; lanes=${mode##*:}
    if [ $st = one ]; then export AZ_SP_ONE_STREAM=1; else unset AZ_SP_ONE_STREAM; fi
    timeout -k 10 200 python -u bench.py $F --sp-lanes $lanes 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['selfplay']; print(json.dumps({'mode':'$mode','games_per_s':s['games_per_s'],'net_wait_s':s['net_wait_s'],'host_s':s['host_s'],'collect_s':s.get('collect_s'),'launch_s':s.get('launch_s')}))" >> gpurun_out/$tag/ab.jsonl
  done
done

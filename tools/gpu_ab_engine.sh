# A/B of the self-play leg: the engine at HEAD (libaz_mcts_base.so, built by hand from
# `git show HEAD:alphazero-gnn_amd/csrc/az_mcts.cpp`) vs the working tree's libaz_mcts.so,
# alternated in one GPU session.   bash tools/gpu_ab_engine.sh <tag>
set -e
tag=${1:-ab_engine}
mkdir -p gpurun_out/$tag
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then export AZ_AB_MCTS_LIB=libaz_mcts_base.so; else unset AZ_AB_MCTS_LIB; fi
    timeout -k 10 200 python -u bench.py $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['selfplay']; print(json.dumps({'lib':'$lib','games_per_s':s['games_per_s'],'net_wait_s':s['net_wait_s'],'host_s':s['host_s'],'assemble_s':s.get('assemble_s'),'collect_s':s.get('collect_s'),'launch_s':s.get('launch_s'),'host_only_gps':s.get('host_only',{}).get('games_per_s')}))" >> gpurun_out/$tag/ab.jsonl
  done
done

# A/B of the bench's self-play leg in one GPU session: base (libaz_hip_base.so) vs the working
# tree's library, alternated.   bash tools/gpu_ab_selfplay.sh <tag>
set -e
tag=${1:-ab_sp}
mkdir -p gpurun_out/$tag
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2; do
  AZ_AB_LIB=libaz_hip_base.so timeout -k 10 200 python -u bench.py $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'lib':'base','games_per_s':d['selfplay']['games_per_s'],'net_wait_s':d['selfplay']['net_wait_s'],'host_s':d['selfplay']['host_s']}))" >> gpurun_out/$tag/ab.jsonl
  timeout -k 10 200 python -u bench.py $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'lib':'new','games_per_s':d['selfplay']['games_per_s'],'net_wait_s':d['selfplay']['net_wait_s'],'host_s':d['selfplay']['host_s']}))" >> gpurun_out/$tag/ab.jsonl
done

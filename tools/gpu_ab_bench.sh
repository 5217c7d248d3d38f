# A/B of the bench's headline step (B = 512) in one GPU session: base (libaz_hip_base.so) vs the
# working tree's library, alternated.   bash tools/gpu_ab_bench.sh <tag>
set -e
tag=${1:-ab_bench}
mkdir -p gpurun_out/$tag
F="--steps 200 --warmup 200 --no-cpu --no-selfplay --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then export AZ_AB_LIB=libaz_hip_base.so; else unset AZ_AB_LIB; fi
    timeout -k 10 200 python -u bench.py $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'lib':'$lib','value':d['value'],'ms_per_step':d['ms_per_step']}))" >> gpurun_out/$tag/ab.jsonl
  done
done

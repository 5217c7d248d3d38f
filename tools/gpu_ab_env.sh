# A/B of the bench's headline step (B = 512) in one GPU session: an env switch off vs on,
# alternated.   bash tools/gpu_ab_env.sh <tag> <VAR>    (A: VAR=1 set, B: unset)
set -e
tag=${1:-ab_env}; var=${2:-AZ_GEMM_NOP2}
mkdir -p gpurun_out/$tag
F="--steps 200 --warmup 200 --no-cpu --no-selfplay --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2 3; do
  for arm in set unset; do
    if [ $arm = set ]; then export $var=1; else unset $var; fi
    timeout -k 10 200 python -u bench.py $F > gpurun_out/$tag/last.json 2> gpurun_out/$tag/last.err
    python -c "import json; d=json.loads(open('gpurun_out/$tag/last.json').read().strip().splitlines()[-1]); print(json.dumps({'$var':'$arm','value':d['value'],'ms_per_step':d['ms_per_step'],'gemm_us':d['roofline']['avg_launch_us']}))" >> gpurun_out/$tag/ab.jsonl
  done
done
unset $var

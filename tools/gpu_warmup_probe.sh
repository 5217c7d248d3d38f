set -e
mkdir -p gpurun_out/wu
F="--no-cpu --no-selfplay --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for cfg in "50 10" "100 20" "200 200" "50 10" "200 200" "500 200"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --steps $1 --warmup $2 $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'steps':$1,'warmup':$2,'value':d['value'],'ms_per_step':d['ms_per_step'],'gemm_us':d['roofline']['avg_launch_us']}))" >> gpurun_out/wu/wu.jsonl
done

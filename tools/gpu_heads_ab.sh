# split-K heads variants in the fused predict_with_gnn step (tuning build: AZ_SPLITK_HEADS_R rows per
# block, AZ_SPLITK_HEADS_MODE), alternated.   bash tools/gpu_heads_ab.sh "B1 B2 ..."
set -e
mkdir -p gpurun_out/heads_ab
for i in 1 2; do
for v in "R=2" "R=1"; do
  export AZ_SPLITK_HEADS_R=${v#*=}
  AZ_TUNING_LIB=1 timeout -k 10 120 python -u tools/presplit_probe.py ${1:-512} | sed "s/^/{\"v\": \"$v\", \"r\": /; s/}$/}}/" >> gpurun_out/heads_ab/probe2.jsonl
done
done
cat gpurun_out/heads_ab/probe2.jsonl

# csk planner miss cost sweep on the P2 self-play GEMM shapes (tuning build, AZ_CSK_MISS), plans
# printed (AZ_CSK_PRINT), alternated twice in one session.   bash tools/gpu_cskmiss.sh
set -e
mkdir -p gpurun_out/cskmiss
for i in 1 2; do
  for m in 0.12 0.3 0.6 1.2 3; do
    AZ_TUNING_LIB=1 AZ_CSK_PRINT=1 AZ_CSK_MISS=$m timeout -k 10 120 python -u tools/p2h_probe.py 800,1576,3150 30 2> gpurun_out/cskmiss/plan_$m.txt | sed "s/^/{\"miss\": $m, \"r\": /; s/}$/}}/" >> gpurun_out/cskmiss/probe.jsonl
  done
done
cat gpurun_out/cskmiss/probe.jsonl
for m in 0.12 0.3 0.6 1.2 3; do echo "== $m"; sort -u gpurun_out/cskmiss/plan_$m.txt | grep csk; done

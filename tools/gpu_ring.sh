# gemm_p3 two- vs three-stage ring (tuning build, AZ_P3_RING), alternated, same session
set -e
mkdir -p gpurun_out/ring
for i in 1 2; do
  for r in 2 3; do
    AZ_TUNING_LIB=1 AZ_P3_RING=$r timeout -k 10 120 python -u tools/p2h_probe.py 512,1024,8192,65536 30 | sed "s/^/{\"ring\": $r, \"r\": /; s/}$/}}/" >> gpurun_out/ring/probe.jsonl
  done
done
cat gpurun_out/ring/probe.jsonl

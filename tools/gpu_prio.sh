# gemm_p3 setprio variants (tuning build, AZ_P3_PRIO = 0 / 1 / 2), alternated, same session
set -e
mkdir -p gpurun_out/prio
for i in 1 2; do
  for r in 0 1 2; do
    AZ_TUNING_LIB=1 AZ_P3_PRIO=$r timeout -k 10 120 python -u tools/p2h_probe.py 512,2048,8192 40 | sed "s/^/{\"prio\": $r, \"r\": /; s/}$/}}/" >> gpurun_out/prio/probe.jsonl
  done
done
cat gpurun_out/prio/probe.jsonl

# 256 x 256 pre-split tile (tuning build, AZ_P3_WIDE=1) vs 256 x 128, alternated; hashes must match
set -e
mkdir -p gpurun_out/wide
for i in 1 2; do
  AZ_TUNING_LIB=1 timeout -k 10 120 python -u tools/p2h_probe.py 8192,16384,65536 10 | sed 's/^/{"wide": 0, "r": /; s/}$/}}/' >> gpurun_out/wide/probe.jsonl
  AZ_TUNING_LIB=1 AZ_P3_WIDE=1 timeout -k 10 120 python -u tools/p2h_probe.py 8192,16384,65536 10 | sed 's/^/{"wide": 1, "r": /; s/}$/}}/' >> gpurun_out/wide/probe.jsonl
done
cat gpurun_out/wide/probe.jsonl

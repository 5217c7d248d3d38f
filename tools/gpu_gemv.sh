set -o pipefail
mkdir -p gpurun_out/gemv
for v in 42 22 82 41 44 12; do
  AZ_GEMV_ROWS=$v timeout -k 10 120 python -u tools/gemv_probe.py >> gpurun_out/gemv/probe.log 2>&1 || exit 1
done

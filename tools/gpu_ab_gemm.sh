# A/B of ops.linear at self-play shapes in one GPU session: base (libaz_hip_base.so) vs the
# working tree's library, alternated.   bash tools/gpu_ab_gemm.sh <tag> [M list]
set -e
tag=${1:-ab_gemm}; Ms=${2:-1576,2048,3086,3150,4096}
mkdir -p gpurun_out/$tag
for i in 1 2; do
  AZ_AB_LIB=libaz_hip_base.so timeout -k 10 120 python -u tools/gemm_ab.py $Ms 20 >> gpurun_out/$tag/ab.jsonl
  timeout -k 10 120 python -u tools/gemm_ab.py $Ms 20 >> gpurun_out/$tag/ab.jsonl
done

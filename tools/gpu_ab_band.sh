# A/B of the band layer in one GPU session: base (libaz_hip_base.so, tools/ab_lib.sh) vs the
# working tree's libaz_hip.so, alternated.   bash tools/gpu_ab_band.sh <tag>
set -e
tag=${1:-ab_band}
mkdir -p gpurun_out/$tag
for i in 1 2; do
  AZ_AB_LIB=libaz_hip_base.so timeout -k 10 100 python -u tools/band_probe.py 512 20 2>/dev/null | sed "s/^/base /" >> gpurun_out/$tag/ab.log
  timeout -k 10 100 python -u tools/band_probe.py 512 20 2>/dev/null | sed "s/^/new  /" >> gpurun_out/$tag/ab.log
done

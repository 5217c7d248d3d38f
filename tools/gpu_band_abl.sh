# Timing ablations of gnn_layer_band_kernel (tuning build; results wrong by design):
#   bash tools/gpu_band_abl.sh <tag>   -> gpurun_out/<tag>/abl.log
set -e
tag=${1:-band_abl}
mkdir -p gpurun_out/$tag
for a in ${ABLS:-0 1 2 4 8 16 15 31}; do
  AZ_TUNING_LIB=1 AZ_BAND_ABL=$a timeout -k 10 100 python -u tools/band_probe.py 512 20 2>/dev/null | sed "s/^/abl=$a /" >> gpurun_out/$tag/abl.log
done

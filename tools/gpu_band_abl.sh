set -e
mkdir -p gpurun_out/r03f
for a in ${ABLS:-0 1 2 4 8 16 15 31}; do
  AZ_TUNING_LIB=1 AZ_BAND_ABL=$a timeout -k 10 100 python -u tools/band_probe.py 512 20 2>/dev/null | sed "s/^/abl=$a /" >> gpurun_out/r03f/abl.log
done

# band layer after the fp16 form: per-phase trace and timing ablations (tuning build)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
AZ_TUNING_LIB=1 AZ_BAND_ABL=256 timeout -k 10 120 python -u tools/band_trace.py 512 > $O/band_trace.txt 2>&1 || { tail -20 $O/band_trace.txt; exit 1; }
cat $O/band_trace.txt
ABLS="0 1 2 4 8 16 31" bash tools/gpu_band_abl.sh r04k_abl || exit 1
cat gpurun_out/r04k_abl/abl.log

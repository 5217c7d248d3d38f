# GPU-box, round 3: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the bench's B = 512
# step and of the band-mode GNN layer (tools/band_probe.py), then the SQ / GRBM counter passes and
# a kernel trace of the band probe (tools/gpu_kernel_pmc.sh).  Summaries:
#   python tools/pmc_summary.py gpurun_out/prof_TAG TAG
#   python tools/pmc_kernel_report.py gpurun_out/kpmc_TAG_band gnn_layer_band
#   bash tools/gpu_pmc_r03.sh TAG
set -u
TAG=${1:-r03}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --no-selfplay --no-train --no-agg-extra --no-grid --no-b1 --large-batch 0"
P="python3 tools/band_probe.py 512 3"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ffetch -o run -- $P > $OUT/ffetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/fwrite -o run -- $P > $OUT/fwrite.log 2>&1 || exit $?
bash tools/gpu_kernel_pmc.sh ${TAG}_band $P || exit $?
bash tools/gpu_kernel_pmc.sh ${TAG}_gemm $B || exit $?
echo done > $OUT/done

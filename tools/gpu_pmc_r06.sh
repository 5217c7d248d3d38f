# GPU-box, round 6: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and SQ / TCC / GRBM
# counters at HEAD's kernels for everything the bench line quotes from profiles/pmc.json:
#   step  -- the B = 512 step (roofline.traffic: the standalone output_transform.0 call) and the
#            band layer (layer_roofline.traffic)
#   csk   -- the self-play GEMM (gemm_x3_csk, pre-split P2 form) at M = 800 / 1,576 / 3,150
#            (gemm_shapes[].committed_pmc) and output_transform.0 at M = 65,536 (large_batch)
# Summaries: python tools/pmc_summary.py gpurun_out/prof_TAG TAG;
#            python tools/csk_pmc_report.py gpurun_out/cskpmc_TAG out.json
#   bash tools/gpu_pmc_r06.sh TAG [step|csk]
set -u
TAG=${1:-r06}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --settle-ms 0 --no-cpu --no-selfplay --no-train --no-agg-extra --no-grid --no-b1 --large-batch 0"
P="python3 tools/band_probe.py 512 3"
PART=${2:-step}
if [ "$PART" = step ]; then
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ffetch -o run -- $P > $OUT/ffetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/fwrite -o run -- $P > $OUT/fwrite.log 2>&1 || exit $?
bash tools/gpu_kernel_pmc.sh ${TAG}_gemm $B || exit $?
fi
if [ "$PART" = csk ]; then
O=gpurun_out/cskpmc_$TAG
for M in 800 1576 3150 65536; do
  D=$O/csk_$M
  mkdir -p $D
  R=20; [ $M -gt 4096 ] && R=3
  C="python3 tools/gemm_ab.py $M $R"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $C > $D/fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $C > $D/write.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/tcc -o run -- $C > $D/tcc.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $D/sq -o run -- $C > $D/sq.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- $C > $D/kt.log 2>&1 || exit 1
done
fi
echo done > $OUT/done_$PART

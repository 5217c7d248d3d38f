# PMC of the self-play GEMM (cycled stream-K on pre-split operands, registered weights) at
# M = 1,576 / 3,150: FETCH / WRITE / TCC+GRBM / SQ passes + a kernel trace, each its own run.
#   bash tools/gpu_csk_pmc_p2.sh TAG;  python tools/csk_pmc_report.py gpurun_out/cskpmc_TAG
set -u
TAG=${1:-r04}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cskpmc_$TAG
for M in 1576 3150; do
  D=$O/csk_$M
  mkdir -p $D
  C="python3 tools/gemm_ab.py $M 20"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $C > $D/fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $C > $D/write.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/tcc -o run -- $C > $D/tcc.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $D/sq -o run -- $C > $D/sq.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- $C > $D/kt.log 2>&1 || exit 1
done
echo done > $O/done

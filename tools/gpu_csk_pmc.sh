# PMC of the self-play GEMM (ops.linear 3136 x 3136 at M) as the product runs it (gemm_x3_csk) and
# as round 3 ran it (tuning build, AZ_CSK=off: gemm_x3_sk): FETCH_SIZE, WRITE_SIZE, TCC hit/miss +
# GRBM, SQ busy counters, kernel trace -- each its own rocprofv3 run.
#   bash tools/gpu_csk_pmc.sh TAG "800 1576 3150"     summary: python tools/csk_pmc_report.py gpurun_out/cskpmc_TAG
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cskpmc_${1:-r04}
mkdir -p $O
for M in ${2:-800 1576 3150}; do
  for cfg in csk sk; do
    if [ $cfg = sk ]; then export AZ_TUNING_LIB=1 AZ_CSK=off; else unset AZ_TUNING_LIB AZ_CSK; fi
    D=$O/${cfg}_$M
    mkdir -p $D
    C="python3 tools/gemm_ab.py $M 20"
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $C > $D/fetch.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $C > $D/write.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/tcc -o run -- $C > $D/tcc.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $D/sq -o run -- $C > $D/sq.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- $C > $D/kt.log 2>&1 || exit 1
  done
done
echo done > $O/done

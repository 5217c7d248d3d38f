# GPU-box: SQ / GRBM / TCC counters of az_gemm_f32 for a list of tile configs at one shape.
#   bash tools/gpu_gemm_pmc.sh TAG "6 16" M [N K]   ("auto" = the dispatcher's own choice)
export AZ_TUNING_LIB=1   # A/B switches live in the tuning build
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; CFGS=$2; M=$3; N=${4:-3136}; K=${5:-3136}
O=gpurun_out/gpmc_$TAG
mkdir -p $O
for c in $CFGS; do
  if [ "$c" = auto ]; then unset AZ_GEMM_CFG; else export AZ_GEMM_CFG=$c; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/c${c}_p1 -o run -- python3 tools/gemm_one.py $M $N $K 20 > $O/c${c}_p1.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/c${c}_p2 -o run -- python3 tools/gemm_one.py $M $N $K 20 > $O/c${c}_p2.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c${c}_kt -o run -- python3 tools/gemm_one.py $M $N $K 20 > $O/c${c}_kt.log 2>&1 || exit $?
done
echo done > $O/done

# GPU-box: SQ / TCC / GRBM counter passes + kernel trace of one command (separate runs, per the
# MICROARCH guide: counters never combined with tracing).
#   bash tools/gpu_kernel_pmc.sh TAG python3 tools/fused_probe.py one
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/kpmc_$TAG
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- "$@" > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p2 -o run -- "$@" > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p3 -o run -- "$@" > $O/p3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- "$@" > $O/kt.log 2>&1 || exit $?
echo done > $O/done

# TA / TCP counters of one command (two passes), then a kernel trace.  bash tools/gpu_ta_pmc.sh TAG cmd...
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/tapmc_$TAG
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p1 -o run -- "$@" > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d $O/p2 -o run -- "$@" > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- "$@" > $O/kt.log 2>&1 || exit $?
echo done > $O/done

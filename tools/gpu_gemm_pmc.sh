set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/gpmc
mkdir -p $O
export AZ_GEMM_CFG=0 AZ_GEMM_STREAMK=0
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- python3 tools/gemm_one.py 512 3136 3136 5 > $O/p1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 tools/gemm_one.py 512 3136 3136 5 > $O/p2.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_F32 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/p3 -o run -- python3 tools/gemm_one.py 512 3136 3136 5 > $O/p3.log 2>&1 || exit $?
echo done > $O/done

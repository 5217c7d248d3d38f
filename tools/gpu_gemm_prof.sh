set -u
TAG=${1:-g}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/gemm_$TAG
mkdir -p $OUT
timeout -k 10 600 python tools/gemm_sweep.py > $OUT/sweep.jsonl 2> $OUT/sweep.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-aggregate > $OUT/pmc1.log 2>&1 || exit $?
echo done > $OUT/done

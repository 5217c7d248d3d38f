# GPU-box: correctness + timing sweep of LDS-DMA GEMM configs: bash tools/gpu_glds.sh TAG CFGS SPLITS
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/glds_$1
mkdir -p $O
timeout -k 10 300 python tools/gemm_sweep.py quickcheck $2 > $O/check.jsonl 2> $O/check.err || exit $?
timeout -k 10 900 python tools/gemm_sweep.py glds $2 $3 > $O/sweep.jsonl 2> $O/sweep.err || exit $?
echo done > $O/done

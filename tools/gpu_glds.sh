# GPU-box: correctness + timing sweep of the LDS-DMA GEMM configs (tools/gemm_sweep.py glds).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/glds_$1
mkdir -p $O
timeout -k 10 300 python tools/gemm_sweep.py quickcheck > $O/check.jsonl 2> $O/check.err || exit $?
timeout -k 10 900 python tools/gemm_sweep.py glds > $O/sweep.jsonl 2> $O/sweep.err || exit $?
echo done > $O/done

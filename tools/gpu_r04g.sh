# row_scale_kernel rewrite: GEMM tests, headline A/B vs HEAD; self-play thread-count / wait-policy A/B
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm or x3 or h3 or streamk or transform or heads" --timeout 300 --timeout-method thread > $O/gemm_tests.log 2>&1 || { tail -30 $O/gemm_tests.log; exit 1; }
tail -2 $O/gemm_tests.log
bash tools/gpu_ab_bench.sh r04g_bench || exit 1
cat gpurun_out/r04g_bench/ab.jsonl
bash tools/gpu_ab_spthreads.sh r04g_sp || exit 1
cat gpurun_out/r04g_sp/ab.jsonl
echo done > $O/done

set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep2
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu > gpurun_out/sweep2/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sweep2/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python tools/gemm_sweep.py > gpurun_out/sweep2/sweep.jsonl 2> gpurun_out/sweep2/sweep.err

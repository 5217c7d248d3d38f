# GPU-box A/B of the stream-K heads finalize (self-play leg): the bench's self-play leg under
# rocprofv3 --kernel-trace --stats per library variant, then the presplit / kernel / trained GPU
# tests on the working tree's library.
#   VARIANTS="base=libaz_hip_base.so new=" bash tools/gpu_r06_csk_finalize_ab.sh
cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0"
for v in ${VARIANTS:-base=libaz_hip_base.so new=}; do
  n=${v%%=*}; l=${v#*=}
  AZ_AB_LIB=$l timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cskfin/$n -o run -- python3 $B > gpurun_out/cskfin_$n.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_presplit.py tests/test_gpu_kernels.py tests/test_gpu_trained.py tests/test_gpu_selfplay.py > gpurun_out/cskfin_pytest.log 2>&1 || exit 1

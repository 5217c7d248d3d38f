# band layer in the fp16 form: its tests, A/B vs the bf16 form; OMP binding A/B; headline trace;
# DP tests
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "band or grid or layer_ot or fused or synth" --timeout 300 --timeout-method thread > $O/band_tests.log 2>&1 || { tail -30 $O/band_tests.log; exit 1; }
tail -2 $O/band_tests.log
bash tools/gpu_ab_band.sh r04f_band || exit 1
cat gpurun_out/r04f_band/ab.log
bash tools/gpu_r04e.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/dist.log 2>&1 || { tail -30 $O/dist.log; exit 1; }
tail -2 $O/dist.log
echo done > $O/done

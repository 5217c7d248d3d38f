# band layer with per-row scales: band tests (incl. the wide-dynamic-range one), A/B vs HEAD
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -k "band or grid or layer_ot or fused or synth or wide" --timeout 300 --timeout-method thread > $O/band_tests.log 2>&1 || { tail -40 $O/band_tests.log; exit 1; }
tail -2 $O/band_tests.log
bash tools/gpu_ab_band.sh ${TAG:-r04r} || exit 1
cat gpurun_out/${TAG:-r04r}/ab.log

set -e
mkdir -p gpurun_out/${TAG:-bandv1}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "band or ot_infer" -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG:-bandv1}/tests.log 2>&1
timeout -k 10 120 python -u tools/band_probe.py 512 20 > gpurun_out/${TAG:-bandv1}/probe.log 2>&1
ABLS="${ABLS:-0 2 16}" bash tools/gpu_band_abl.sh ${TAG:-bandv1}

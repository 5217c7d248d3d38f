set -o pipefail
mkdir -p gpurun_out/r02j
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "linear or transform or heads" > gpurun_out/r02j/t.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-selfplay --no-train --no-cpu --no-grid --no-b1 --large-batch 0 > gpurun_out/r02j/bench.json 2> gpurun_out/r02j/bench.err && \
AZ_TUNING_LIB=1 AZ_GEMM_NO_KSLICE=1 timeout -k 10 400 python -u bench.py --no-selfplay --no-train --no-cpu --no-grid --no-b1 --large-batch 0 > gpurun_out/r02j/bench_noks.json 2> gpurun_out/r02j/bench_noks.err

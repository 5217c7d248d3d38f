# arena speculative batches: parity tests, arena legs, per-call latency and its kernel split
set -o pipefail
mkdir -p gpurun_out/r02h
export AZ_REPORT_DIR=gpurun_out/r02h
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_selfplay.py tests/test_gpu_wrappers.py > gpurun_out/r02h/t.log 2>&1 && \
timeout -k 10 300 python -u tools/arena_bench.py 4 > gpurun_out/r02h/arena.log 2>&1 && \
timeout -k 10 200 python -u tools/latency_probe.py > gpurun_out/r02h/lat.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02h/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/latency_probe.py 300 > $GRAFT_REPO_ROOT/gpurun_out/r02h/kt.log 2>&1

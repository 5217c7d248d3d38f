# one-launch leaf (serial GEMV form): wrapper + selfplay tests, b1 leg, host probe, arena bench
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-leaf2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wrappers.py -x -q --timeout 300 --timeout-method thread > $O/wrappers.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfplay.py -x -q --timeout 300 --timeout-method thread > $O/selfplay.log 2>&1 || exit $?
bash tools/gpu_b1.sh ${1:-leaf2}/b1 || exit $?
timeout -k 10 300 python -u tools/b1_host_probe.py 3000 > $O/probe.json 2> $O/probe.err || exit $?
timeout -k 10 400 python -u tools/arena_bench.py 4 > $O/arena.json 2> $O/arena.err || exit $?
echo done > $O/done

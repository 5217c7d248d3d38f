# GPU-box: the one-launch batch-1 leaf -- wrapper tests, then the bench's b1 leg + kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-leaf}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wrappers.py -x -q --timeout 300 --timeout-method thread > $O/wrappers.log 2>&1 || exit $?
bash tools/gpu_b1.sh ${1:-leaf}/b1 || exit $?
echo done > $O/done

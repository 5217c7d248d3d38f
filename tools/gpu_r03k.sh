# GPU-box: the one-launch batch-1 leaf (wrapper tests, then the bench's b1 leg + kernel stats),
# then self-play with per-lane streams (profile + the self-play GPU tests).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wrappers.py -x -q --timeout 300 --timeout-method thread > $O/wrappers.log 2>&1 || exit $?
bash tools/gpu_b1.sh ${1:-r03k}/b1 || exit $?
timeout -k 10 600 python -u tools/selfplay_gpu_profile.py 4096 > $O/sp_prof.txt 2> $O/sp_prof.err || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_selfplay.py -x -q --timeout 300 --timeout-method thread > $O/selfplay_tests.log 2>&1 || exit $?
echo done > $O/done

# leaf kernel weight-stream experiments (tuning build): trace per AZ_LEAF_MODE, then the product
# path's wrapper tests and b1 leg
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-leafm}
mkdir -p $O
for m in ${LEAF_MODES:-0 3}; do
  AZ_LEAF_MODE=$m timeout -k 10 200 python -u tools/leaf_probe.py 40 > $O/trace_$m.json 2> $O/trace_$m.err || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_wrappers.py -x -q --timeout 300 --timeout-method thread > $O/wrappers.log 2>&1 || exit $?
bash tools/gpu_b1.sh ${1:-leafm}/b1 || exit $?
echo done > $O/done

# GPU-box: the VALU lane exchanges (bitwise probe), the heads / trunk GPU tests, and the trunk's
# three forms + one self-play round at self-play sizes under a kernel trace.
#   bash tools/gpu_r06_heads.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06h}
mkdir -p $O
timeout -k 10 60 ./tools/probes/wave_xor_probe > $O/wave_xor_probe.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_presplit.py tests/test_gpu_kernels.py tests/test_gpu_selfplay.py -k "trunk or heads or presplit or c4_gnn_eval or predict_both or batch_rows" \
  > $O/pytest.log 2>&1 || exit $?
export TMPDIR=/tmp
for B in 1576 3150; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tv$B -o run -- python3 tools/trunk_variants_probe.py $B 30 > $O/tv$B.log 2>&1 || exit 1
done

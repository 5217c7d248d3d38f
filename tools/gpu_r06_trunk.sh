# GPU-box: round-6 trunk check after the packed-FP32 fix -- the self-check probe at two blocks per
# CU (NB 1..3, libaz_hip_exp.so = az_trunk.hip with -DAZ_TUNING -DAZ_TRUNK_SELFCHECK linked with the
# tuning objects), the trunk / hand-off GPU tests, and the NB sweep for the rounds model.
#   bash tools/gpu_r06_trunk.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/${1:-r06trunk}; mkdir -p $R
for nb in 1 2 3; do
  AZ_AB_LIB=libaz_hip_exp.so AZ_TUNING_LIB=1 AZ_TRUNK_NB=$nb timeout -k 10 120 \
    python tools/trunk_selfcheck_probe.py 512,1576,3150 >> $R/selfcheck.txt 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_presplit.py tests/test_gpu_kernels.py -k "trunk or presplit or c4_gnn_eval" \
  > $R/pytest.log 2>&1 || exit $?
BS=256,512,768,1024,1576,2048,2560,3150,4096
timeout -k 10 120 python tools/trunk_w2f_probe.py $BS >> $R/nb_sweep.txt 2>&1 || exit $?
for nb in 1 2 3 4 5 6 7 8; do
  AZ_TUNING_LIB=1 AZ_TRUNK_NB=$nb timeout -k 10 120 python tools/trunk_w2f_probe.py $BS >> $R/nb_sweep.txt 2>&1 || exit $?
done

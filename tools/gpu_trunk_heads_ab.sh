# GPU-box: predict_both's standard heads in the split-A trunk (trunk_rows_heads) -- the GPU tests
# that cover it, then the self-play leg with and without it (AZ_NO_TRUNK_HEADS, tuning build),
# alternating, same session.   bash tools/gpu_trunk_heads_ab.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/${1:-th}; mkdir -p $R
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selfplay.py tests/test_gpu_presplit.py tests/test_gpu_trained.py > $R/pytest.log 2>&1 || exit $?
export AZ_TUNING_LIB=1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0 > $R/sp_fused_$i.json 2>> $R/err.txt || exit $?
  AZ_NO_TRUNK_HEADS=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0 > $R/sp_sep_$i.json 2>> $R/err.txt || exit $?
done

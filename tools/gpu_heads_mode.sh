# GPU-box: GPU tests + smoke, then A/B of the split-K heads tail: one launch per row (default)
# with R = 1/2/4 rows per block vs one row per block vs chunk partials + finalize, B = 512 step.
export AZ_TUNING_LIB=1   # A/B switches live in the tuning build
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh hm || exit $?
Q="--no-cpu --no-selfplay --no-train --no-aggregate --no-grid --large-batch 0"
for r in 1 2; do
  for m in w1 w2 w4 rows chunks; do
    AZ_SPLITK_HEADS_R=${m:1:1} AZ_SPLITK_HEADS_MODE=$m timeout -k 10 120 python bench.py --steps 200 --warmup 20 $Q > gpurun_out/hm_$m.json 2>/dev/null || exit $?
    python -c "import json;d=json.load(open('gpurun_out/hm_$m.json'));print('$m', d['value'], d['ms_per_step'])"
  done
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hm_kt -o run -- python3 bench.py --steps 50 --warmup 5 $Q > gpurun_out/hm_kt.log 2>&1 || exit $?

# GPU-box A/B of splitk_heads_partial_kernel rows per block (AZ_SPLITK_HEADS_ROWS = 16 / 8 / 4):
# bench main step only, plus a kernel-trace pass per setting.   bash tools/heads_rows_probe.sh
export AZ_TUNING_LIB=1   # A/B switches live in the tuning build
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/hrows
mkdir -p $O
Q="--no-cpu --no-selfplay --no-train --no-aggregate --no-grid --large-batch 0"
for r in 16 8 4 16 8 4; do
  AZ_SPLITK_HEADS_ROWS=$r timeout -k 10 120 python bench.py --steps 200 --warmup 20 $Q > $O/b$r.json 2> $O/b$r.err || exit $?
  python -c "import json;d=json.load(open('$O/b$r.json'));print($r, d['value'], d['ms_per_step'])"
done
for r in 16 8 4; do
  AZ_SPLITK_HEADS_ROWS=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$r -o run -- python3 bench.py --steps 50 --warmup 5 $Q > $O/kt$r.log 2>&1 || exit $?
  grep -h 'splitk_heads\|finalize' $O/kt$r/run_kernel_stats.csv | cut -d, -f1-4
done

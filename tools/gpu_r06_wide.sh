# GPU-box: the 256 x 256 pre-split tile with split-K (tuning build, AZ_P3_WIDE=1,
# AZ_P3_WIDE_SPLITS=S) vs the product's 256 x 128 tile at M = 512: ops.linear time per call and
# the kernel-trace averages.   bash tools/gpu_r06_wide.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-wide}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prod -o run -- python3 tools/p2h_probe.py 512 100 > $O/prod.log 2>&1 || exit 1
for S in 4 6 8 9; do
  AZ_TUNING_LIB=1 AZ_P3_WIDE=1 AZ_P3_WIDE_SPLITS=$S timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w$S -o run -- python3 tools/p2h_probe.py 512 100 > $O/w$S.log 2>&1 || exit 1
done
echo done > $O/done

set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06f}
mkdir -p $O
for M in ${SP_M:-1576 3150}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/m$M -o run -- python3 tools/sp_round_probe.py $M 50 > $O/m$M.log 2>&1 || exit 1
done
for B in 1576 3150; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tv$B -o run -- python3 tools/trunk_variants_probe.py $B 30 > $O/tv$B.log 2>&1 || exit 1
done

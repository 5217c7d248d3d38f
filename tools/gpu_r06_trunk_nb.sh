# GPU-box: the split-A trunk (c4_gnn_eval) and the trunk + standard heads (predict_both) per
# boards-per-block choice (tuning build, AZ_TRUNK_NB; "m" = the rounds model) at B = 512 /
# 1,576 / 3,150: kernel-trace averages.   bash tools/gpu_r06_trunk_nb.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-tnb}
mkdir -p $O
for B in 512 1576 3150; do
  for nb in m 1 2 3; do
    C="timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b${B}_nb$nb -o run -- python3 tools/trunk_variants_probe.py $B 30"
    if [ $nb = m ]; then AZ_TUNING_LIB=1 $C > $O/b${B}_nb$nb.log 2>&1 || exit 1
    else AZ_TUNING_LIB=1 AZ_TRUNK_NB=$nb $C > $O/b${B}_nb$nb.log 2>&1 || exit 1; fi
  done
done
echo done > $O/done

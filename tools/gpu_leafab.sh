# leaf kernel A/B (tuning build, untraced): the b1 leg's predict_both latency per AZ_LEAF_MODE,
# interleaved twice
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-leafab}
mkdir -p $O
for rep in 1 2; do
  for m in 0 1 2; do
    AZ_TUNING_LIB=1 AZ_LEAF_MODE=$m timeout -k 10 200 python -u tools/b1_host_probe.py 3000 > $O/probe_${m}_$rep.json 2> $O/probe_${m}_$rep.err || exit $?
  done
done
echo done > $O/done

# pre-split tile timing ablations (tuning build, AZ_P3_ABL: 1 no epilogue stores, 2 no MFMAs,
# 4 no DMA; 5 / 6 combinations): kernel-trace averages of gemm_p3 at M = 512 and 8,192
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/p3abl
mkdir -p $O
for abl in ${ABLS:-0 1 2 4 5 6}; do
  for M in 512 8192; do
    AZ_TUNING_LIB=1 AZ_P3_ABL=$abl timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/a${abl}_m$M -o run -- python3 tools/p2h_probe.py $M 40 > $O/a${abl}_m$M.log 2>&1 || exit 1
    python3 - $O/a${abl}_m$M/run_kernel_stats.csv $abl $M <<'PY'
import csv, json, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm_p3" in r["Name"] or "gemm_x3_csk" in r["Name"]:
        print(json.dumps({"abl": int(sys.argv[2]), "M": int(sys.argv[3]), "kernel": r["Name"][:40], "avg_us": round(float(r["AverageNs"]) / 1e3, 2), "calls": int(r["Calls"])}))
PY
  done
done

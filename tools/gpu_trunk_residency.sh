# GPU-box: tools/trunk_residency_probe.py over NB x extra dynamic LDS on the experiment library
#   bash tools/gpu_trunk_residency.sh TAG "NB list" "DYN list" [B,B,...]
# The library (built here, on the CPU side, after the tuning build): az_trunk.hip with
# -DAZ_TUNING -DAZ_TRUNK_SMALL_UNION (two trunk blocks fit a CU) linked with the other tuning objects:
#   cd alphazero-gnn_amd/csrc && hipcc <build.py FLAGS> -DAZ_TUNING -DAZ_TRUNK_SMALL_UNION \
#     -c az_trunk.hip -o /tmp/az_trunk.o && hipcc --offload-arch=gfx950 -shared -fPIC \
#     -o ../azhip/libaz_hip_exp.so $(ls build/tuning/*.o | grep -v az_trunk.o) /tmp/az_trunk.o
set -u
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/${1:-resid}; mkdir -p $R
export AZ_AB_LIB=${AZ_AB_LIB:-libaz_hip_exp.so} AZ_TUNING_LIB=1
for nb in ${2:-1 2}; do
  for dyn in ${3:-0 4096 100000}; do
    AZ_TRUNK_NB=$nb AZ_TRUNK_DYN_LDS=$dyn timeout -k 10 120 python tools/trunk_residency_probe.py ${4:-512,1576,3150} >> $R/probe.txt 2>&1 || exit $?
  done
done

# Build alphazero-gnn_amd/azhip/libaz_hip_base.so: the product library with the listed csrc
# files taken at git revision REV (default HEAD), everything else as in the working tree -- the
# "before" side of an A/B timing run (AZ_AB_LIB=libaz_hip_base.so selects it).
#   bash tools/ab_lib.sh [REV] file.hip ...
set -e
REV=${1:-HEAD}; shift
cd "$(dirname "$0")/.."
B=alphazero-gnn_amd/csrc_ab; rm -rf $B; mkdir -p $B   # same depth: "../../include"
cp alphazero-gnn_amd/csrc/*.hip alphazero-gnn_amd/csrc/*.h $B/
for f in "$@"; do git show $REV:alphazero-gnn_amd/csrc/$f > $B/$f; done
objs=""
for f in $B/*.hip; do
  o=$B/$(basename $f .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function \
    -fno-gpu-rdc -Xclang -target-feature -Xclang -packed-fp32-ops -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-z,defs -o alphazero-gnn_amd/azhip/libaz_hip_base.so $objs
rm -rf $B
echo built alphazero-gnn_amd/azhip/libaz_hip_base.so

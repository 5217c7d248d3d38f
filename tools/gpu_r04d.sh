# GPU suite + bench (driver's command) + the native engine's thread scaling on this host
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04d}
mkdir -p $O
g++ -O3 -std=c++17 -fopenmp -ffp-contract=off tools/native/mcts_prof.cpp alphazero-gnn_amd/csrc/az_mcts.cpp -o /tmp/mcts_prof || exit 1
for t in 2 4 8 16; do timeout -k 10 120 /tmp/mcts_prof 2048 $t >> $O/mcts_scaling.txt || exit 1; done
for t in 2 16; do OMP_PROC_BIND=close OMP_PLACES=cores timeout -k 10 120 /tmp/mcts_prof 2048 $t | sed 's/^/close-cores /' >> $O/mcts_scaling.txt || exit 1; done
lscpu > $O/lscpu.txt 2>&1
nproc >> $O/lscpu.txt
bash tools/gpu_round4.sh $1 tests

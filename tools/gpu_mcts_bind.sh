# Native MCTS engine thread scaling on the GPU box's host, default placement vs OpenMP binding
#   bash tools/gpu_mcts_bind.sh   (tools/native/mcts_prof.bin built beforehand)
set -e
mkdir -p gpurun_out/mpb
for t in 2 8 16; do
  timeout -k 5 120 ./tools/native/mcts_prof.bin 2048 $t | sed "s/^/default /" >> gpurun_out/mpb/bind.txt
  OMP_PROC_BIND=spread OMP_PLACES=cores timeout -k 5 120 ./tools/native/mcts_prof.bin 2048 $t | sed "s/^/spread-cores /" >> gpurun_out/mpb/bind.txt
  OMP_PROC_BIND=close OMP_PLACES=cores timeout -k 5 120 ./tools/native/mcts_prof.bin 2048 $t | sed "s/^/close-cores /" >> gpurun_out/mpb/bind.txt
done
nproc >> gpurun_out/mpb/bind.txt

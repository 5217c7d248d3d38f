# OMP binding A/B of the self-play leg + a kernel trace of the B = 512 headline step
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
bash tools/gpu_ab_ompbind.sh r04e_omp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 200 --warmup 200 --no-cpu --no-selfplay --no-train --no-b1 --no-grid --no-aggregate --large-batch 0 > $O/prof_bench.json 2> $O/prof.err || exit 1
echo done > $O/done

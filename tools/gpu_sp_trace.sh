# Kernel + memory-copy trace of the bench's self-play leg alone (timeline analysis:
# tools/sp_timeline.py).   bash tools/gpu_sp_trace.sh <tag>
set -e
tag=${1:-sp_trace}
O=gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o run -- python3 bench.py $F > $O/bench.json 2> $O/prof.err
python tools/sp_timeline.py $O/prof > $O/timeline.txt
cat $O/timeline.txt

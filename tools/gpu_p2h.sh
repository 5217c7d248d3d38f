# fp16-form GEMM on pre-split planes vs splitting in the tile (tuning build), two rounds, plus a
# kernel-stats pass of each.   bash tools/gpu_p2h.sh <tag>
set -e
tag=${1:-p2h}
O=gpurun_out/$tag
mkdir -p $O
export AZ_TUNING_LIB=1 AZ_P3_REUSE=1 TMPDIR=/tmp
for i in 1 2; do
  for t in 1 16; do
    AZ_GEMM_X3=$t timeout -k 10 120 python -u tools/p2h_probe.py 512,1576,4096 50 >> $O/probe.jsonl 2>> $O/probe.err
  done
done
for t in 1 16; do
  AZ_GEMM_X3=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$t -o run -- python3 tools/p2h_probe.py 512,4096 50 > $O/kt$t.log 2>&1
done
cat $O/probe.jsonl

# gemm_p3 (x3 GEMM on pre-split planes, LDS-DMA staged) vs gemm_x3: correctness on small shapes,
# then timing (AZ_P3_REUSE=1: the planes are split on the first call only, so the events time the
# tile kernel + its reduce alone).   bash tools/gpu_p3.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-p3}
O=gpurun_out/$T
mkdir -p $O
export AZ_TUNING_LIB=1
timeout -k 10 300 python tools/gemm_sweep.py x3 "100:200:96,37:1001:1024,300:256:1024,512" 15 auto,1,3 > $O/check.jsonl 2> $O/check.err || exit $?
timeout -k 10 600 python tools/gemm_sweep.py x3 "${P3_MS:-512,800,1576,4096}" 1,15 auto > $O/sweep.jsonl 2> $O/sweep.err || exit $?
AZ_P3_REUSE=1 timeout -k 10 600 python tools/gemm_sweep.py x3 "${P3_MS:-512,800,1576,4096}" 15 auto > $O/reuse.jsonl 2> $O/reuse.err || exit $?
AZ_P3_REUSE=1 AZ_P3_SK=1 timeout -k 10 600 python tools/gemm_sweep.py x3 "${P3_MS:-512,800,1576,4096}" 15 auto > $O/reuse_sk.jsonl 2> $O/reuse_sk.err || exit $?
echo done > $O/done

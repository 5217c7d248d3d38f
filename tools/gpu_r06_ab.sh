# GPU-box A/B of library variants in one session (alternating, two rounds): ops.linear at
# M = 512 / 800 / 1,576 / 3,150 (time, error vs float64, output hash -- equal hashes = same bits)
# and the bench's B = 512 step + self-play leg, then the GEMM / presplit / trained GPU tests on
# the working tree's library.  VARIANTS: name=lib pairs (lib "" = libaz_hip.so).
#   VARIANTS="base=libaz_hip_base.so new= d1=libaz_hip_exp.so" bash tools/gpu_r06_ab.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}
mkdir -p $O
V=${VARIANTS:-"base=libaz_hip_base.so new="}
P="python -u tools/p2h_probe.py 512,800,1576,3150 100"
B="python bench.py --steps 200 --warmup 20 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0"
for i in 1 2; do
  for v in $V; do
    n=${v%%=*}; l=${v#*=}
    AZ_AB_LIB=$l timeout -k 10 180 $P > $O/p2h_${n}_$i.jsonl 2>&1 || exit 1
  done
done
for i in 1 2; do
  for v in $V; do
    n=${v%%=*}; l=${v#*=}
    AZ_AB_LIB=$l timeout -k 10 300 $B > $O/bench_${n}_$i.log 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_presplit.py tests/test_gpu_kernels.py tests/test_gpu_trained.py > $O/pytest.log 2>&1 || exit 1
echo done > $O/done

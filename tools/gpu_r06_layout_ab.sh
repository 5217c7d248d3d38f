# GPU-box A/B of the P2 GEMM's row-interleaved planes + three-stage ring (round 6) against the
# previous commit's library (libaz_hip_base.so from tools/ab_lib.sh), in one session:
# ops.linear at M = 512 / 800 / 1,576 / 3,150 (time, error vs float64, output hash -- the hashes
# must agree), the bench's B = 512 step and self-play leg, then the GEMM / presplit GPU tests.
#   bash tools/ab_lib.sh HEAD az_gemm.hip az_trunk.hip az_x3.h && bash tools/gpu_r06_layout_ab.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-layout_ab}
mkdir -p $O
P="python -u tools/p2h_probe.py 512,800,1576,3150 100"
for i in 1 2; do
  AZ_AB_LIB=libaz_hip_base.so timeout -k 10 180 $P > $O/p2h_base_$i.jsonl 2>&1 || exit 1
  timeout -k 10 180 $P > $O/p2h_new_$i.jsonl 2>&1 || exit 1
  AZ_TUNING_LIB=1 AZ_P3_RING=2 timeout -k 10 180 $P > $O/p2h_ring2_$i.jsonl 2>&1 || exit 1
done
B="python bench.py --steps 200 --warmup 20 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0"
for i in 1 2; do
  AZ_AB_LIB=libaz_hip_base.so timeout -k 10 300 $B > $O/bench_base_$i.log 2>&1 || exit 1
  timeout -k 10 300 $B > $O/bench_new_$i.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_presplit.py tests/test_gpu_kernels.py tests/test_gpu_trained.py > $O/pytest.log 2>&1 || exit 1
echo done > $O/done

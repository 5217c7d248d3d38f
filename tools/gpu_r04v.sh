# P2 GEMM (pre-split planes in the product dispatch): GEMM / heads / wrapper tests, bit-identity
# and time vs the in-tile split (tuning build, AZ_GEMM_NOP2=1), headline and self-play A/B vs HEAD
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wrappers.py tests/test_gpu_kernel_variants.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python -u tools/p2h_probe.py 512,800,1576,3150,4096 50 | sed 's/^/p2 /' >> $O/probe.log 2>&1 || exit 1
  AZ_TUNING_LIB=1 AZ_GEMM_NOP2=1 timeout -k 10 120 python -u tools/p2h_probe.py 512,800,1576,3150,4096 50 | sed 's/^/intile /' >> $O/probe.log 2>&1 || exit 1
done
cat $O/probe.log
bash tools/gpu_ab_bench.sh r04v_bench || exit 1
cat gpurun_out/r04v_bench/ab.jsonl
echo done > $O/done

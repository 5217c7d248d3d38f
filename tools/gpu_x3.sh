# gemm_x3 (fp32 on the bf16 matrix cores): correctness on small shapes first, then the sweep.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/x3
export AZ_TUNING_LIB=1
timeout -k 10 400 python tools/gemm_sweep.py x3 "${X3_M0:-100,37:1001:1028,300:256:1024}" 1,2,3 auto,3 > gpurun_out/x3/check.jsonl 2> gpurun_out/x3/check.err || exit $?
timeout -k 10 600 python tools/gemm_sweep.py x3 "${X3_MS:-512,800,128,4096}" "${X3_TILES:-1,2,3}" "${X3_SPLITS:-auto,1,2,3,4,6}" > gpurun_out/x3/sweep.jsonl 2> gpurun_out/x3/sweep.err

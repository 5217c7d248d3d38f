# weighted stream-K + tail skip: x3 tests, GEMM timing at the self-play shapes, one self-play
# round in isolation (kernel stats), then the self-play leg profile
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-sk}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "x3 or transform_heads" --timeout 300 --timeout-method thread > $O/x3_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/gemm_sweep.py x3 "512,700,800,1100,1576,2048" 1 auto > $O/gemm.jsonl 2> $O/gemm.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/spr -o run -- python3 tools/sp_round_probe.py 1576 50 > $O/spr.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/selfplay_gpu_profile.py 4096 > $O/sp_prof.txt 2> $O/sp_prof.err || exit $?
echo done > $O/done

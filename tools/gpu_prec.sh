# x3 vs h3 GEMM forms (tools/prec_probe.py) + the x3/h3 accuracy tests
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-prec}
mkdir -p $O
timeout -k 10 600 python -u tools/prec_probe.py ${2:-512,800,1576,3150,4096} ${3:-1} > $O/prec.jsonl 2> $O/prec.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "x3 or streamk or transform_heads or linear" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo done > $O/done

# Cycled stream-K A/B (tools/csk_probe.py, tuning build): plans vs gemm_x3_sk at self-play M
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-csk}
mkdir -p $O
SPEC=${2:-"1536:off;auto;5,8,0,0;25,42,0,0;1,1,0,0|1280:off;auto;5,10,0,0|1576:off;auto;5,7,1,3;25,39,13,22|3150:off;auto|800:off;auto|2048:off;auto"}
timeout -k 10 900 python -u tools/csk_probe.py "$SPEC" ${3:-1} > $O/csk.jsonl 2> $O/csk.err || exit $?
echo done > $O/done

# GPU-box: GPU tests, then the self-play throughput sweep (tools/sp_sweep.py).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sp_$1
mkdir -p $O
timeout -k 10 900 python -m pytest tests -q -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 python tools/sp_sweep.py > $O/sweep.jsonl 2> $O/sweep.err || exit $?
echo done > $O/done

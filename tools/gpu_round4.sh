# GPU suite + the driver's bench command (+ optional rocprofv3 kernel stats of the bench)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04}
mkdir -p $O
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sp = d.get("selfplay") or {}
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
print("gemm_shapes", d.get("gemm_shapes"))
print("selfplay", sp.get("games_per_s"), "net_wait", sp.get("net_wait_s"), "host", sp.get("host_s"), "agreement", (sp.get("agreement") or {}).get("move_agreement"))
print("layer", (d.get("layer_roofline") or {}).get("avg_launch_us"), "grid", (d.get("grid_forward") or {}).get("ms_per_forward"))
PY
if [ "${3:-}" = "prof" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof_bench.json 2> $O/prof.err || exit 1
fi
echo done > $O/done

# GPU-box, round 4 evidence: the whole -m gpu suite, smoke(), the band probe, the driver's bench
# command and a kernel-stats pass of the B = 512 step, each step under its own limit; the first
# failure ends it.   bash tools/gpu_r04.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r04}
O=gpurun_out/$T
mkdir -p $O
export AZ_REPORT_DIR=$O/reports
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --durations=30 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 200 python -u tools/band_probe.py 512 20 > $O/band_probe.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sp = d.get("selfplay") or {}
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"], "cpu", d["cpu_baseline"]["value"])
print("selfplay", sp.get("games_per_s"), "net_wait", sp.get("net_wait_s"), "host", sp.get("host_s"), "cpu", (sp.get("cpu_baseline") or {}).get("by_threads"))
print("layer", (d.get("layer_roofline") or {}).get("avg_launch_us"), "grid", (d.get("grid_forward") or {}).get("ms_per_forward"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-selfplay --no-train --no-agg-extra --large-batch 0 > $O/kt.log 2>&1 || exit 1
echo done > $O/done

"""The CPU baselines (bench.py cpu_baselines_child, a fresh process on the visible mask) at
several torch thread counts: where the batch-1 self-play loop and the B = 512 forward land on
this host.   python tools/cpu_baseline_threads.py 1,4,8,16 [seconds]   (one JSON line per count)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
threads = [int(t) for t in sys.argv[1].split(",")]
sec = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
cpus = sorted(os.sched_getaffinity(0))
for t in threads:
    spec = {"cpus": cpus, "seconds": sec, "B": 512, "sims": 100, "selfplay": True,
            "grid_seconds": 0, "threads": t}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-baselines-child",
                        json.dumps(spec)], env=dict(os.environ, OMP_NUM_THREADS=str(t)),
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        print(json.dumps({"threads": t, "error": r.stderr[-500:]}), flush=True)
        continue
    d = json.loads(r.stdout.strip().splitlines()[-1])
    sp = d["selfplay"]
    print(json.dumps({"threads": t, "host": d["host"],
                      "gnn_b512_boards_per_s": round(d["gnn_b512"]["value"], 1),
                      "cnn_b512_boards_per_s": round(d["cnn_b512"]["value"], 1),
                      "selfplay_moves_per_s": round(sp["moves"] / sp["seconds"], 3),
                      "selfplay_moves": sp["moves"], "selfplay_seconds": sp["seconds"]}),
          flush=True)

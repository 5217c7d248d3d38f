"""Where the self-play leg's main-thread time goes with the real network on the GPU: the bench's
selfplay_leg under cProfile (tottime), then the leg's stats line.
  python tools/selfplay_gpu_profile.py [games] [threads]"""
import cProfile
import json
import os
import pstats
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))

import bench  # noqa: E402
import hostcpu  # noqa: E402
from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict  # noqa: E402

PIN = hostcpu.pin_rank_to_gpu_numa(0)     # as bench.py, before anything touches the GPU
games = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
threads = int(sys.argv[2]) if len(sys.argv) > 2 else hostcpu.threads_per_rank()
W = synthetic_state_dict(connect4_net_spec(7), 1)
G = synthetic_state_dict(gnn_spec(3136, 2), 2)
args = SimpleNamespace(sp_games=games, sp_sims=100, sp_threads=threads, sp_lanes=2, sp_check=0)
bench.selfplay_leg(W, G, SimpleNamespace(**{**vars(args), "sp_games": 256}), None, 0)   # warm
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
dt, sp = bench.selfplay_leg(W, G, args, None, 0)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
sp.update(games_per_s=round(sp["games"] / dt, 2), seconds=round(dt, 2), threads=threads,
          numa_pin=PIN)
print(json.dumps(sp), flush=True)

"""Self-play throughput sweep on the GPU box: games/s of the native lock-step driver for
several (games, lanes, threads) settings.  python tools/sp_sweep.py [sims]"""
import json
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))

import bench  # noqa: E402
from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict  # noqa: E402

sims = int(sys.argv[1]) if len(sys.argv) > 1 else 100
# optional argv[2]: "games:lanes:threads,..." (default: the round-2 grid)
grid = [tuple(int(v) for v in c.split(":")) for c in sys.argv[2].split(",")] \
    if len(sys.argv) > 2 else None
W = synthetic_state_dict(connect4_net_spec(7), 1)
G = synthetic_state_dict(gnn_spec(3136, 2), 2)
for games, lanes, threads in grid or [(256, 1, 16), (512, 1, 16), (512, 2, 16), (1024, 2, 16),
                                      (2048, 2, 16), (2048, 3, 16), (4096, 2, 16), (2048, 2, 32)]:
    args = SimpleNamespace(sp_games=games, sp_sims=sims, sp_threads=threads, sp_lanes=lanes,
                           sp_check=0)
    t = time.perf_counter()
    dt, sp = bench.selfplay_leg(W, G, args, None, 0)
    sp.update(games_per_s=round(sp["games"] / dt, 2), seconds=round(dt, 2), lanes=lanes,
              threads=threads, wall=round(time.perf_counter() - t, 1))
    print(json.dumps(sp), flush=True)

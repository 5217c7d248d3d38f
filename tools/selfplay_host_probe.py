"""Host-side cost of lock-step native self-play with the network replaced by a constant stub
(CPU only): where the non-GPU time of the self-play leg goes.  cProfile summary + JSON line."""
import cProfile
import json
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from types import SimpleNamespace  # noqa: E402

import selfplay  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402


class StubNet:
    """predict_both with a fixed slightly non-uniform policy and value 0.01 (no GPU)."""

    def __init__(self, A):
        self.pi = (np.arange(A, dtype=np.float32) + 1) / (A * (A + 1) / 2)

    def predict_both(self, boards):
        n = len(boards)
        pi = np.broadcast_to(self.pi, (n, len(self.pi))).copy()
        v = np.full(n, 0.01, np.float32)
        return pi, v, pi, v


games = int(sys.argv[1]) if len(sys.argv) > 1 else 256
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
game = Connect4Game(7)
args = SimpleNamespace(numMCTSSims=100, cpuct=1.0, use_gnn=True, expand_by=5, tempThreshold=15)
net = StubNet(game.getActionSize())
seeds = selfplay.episode_seeds(1234, range(games))
stats = {}
prof = os.environ.get("AZ_PROBE_PROFILE", "1") != "0"
pr = cProfile.Profile()
t0 = time.perf_counter()
if prof:
    pr.enable()
res = selfplay.play_episodes_engine(game, net, args, range(games), seeds, parallel_games=games,
                                    threads=threads, stats=stats)
dt = time.perf_counter() - t0
moves = sum(len(r[0]) for r in res.values()) // 2
if prof:
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
print(json.dumps({"games": games, "threads": threads, "seconds": round(dt, 3),
                  "games_per_s": round(games / dt, 2), "moves": moves,
                  **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in stats.items()}}))

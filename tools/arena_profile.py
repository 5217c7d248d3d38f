"""Where an arena game's time goes (Coach.py:137-145 gating, Connect4 7x7 GNN, 100 sims):
network calls (batch-1 predict_both hipGraph replay + sync) vs the native search, and the raw
replay latency of the batch-1 graph in a tight loop.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from types import SimpleNamespace  # noqa: E402

import selfplay  # noqa: E402
from Arena import Arena  # noqa: E402
from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402
from mcts_native import ArenaPlayer  # noqa: E402

games = int(sys.argv[1]) if len(sys.argv) > 1 else 6
args = SimpleNamespace(numMCTSSims=100, cpuct=1.0, use_gnn=True, dropout=0.3, gnn_layers=2)
game = Connect4Game(7)
torch.manual_seed(0)
pnet, nnet = Connect4GNNWrapper(game, args), Connect4GNNWrapper(game, args)

stat = {"calls": 0, "net_s": 0.0}
orig = selfplay._net_call


def timed_call(net, boards, want_gnn):
    t0 = time.perf_counter()
    r = orig(net, boards, want_gnn)
    stat["net_s"] += time.perf_counter() - t0
    stat["calls"] += 1
    return r


selfplay._net_call = timed_call
np.random.seed(7)
p1, p2 = ArenaPlayer(game, pnet, args), ArenaPlayer(game, nnet, args)
t0 = time.perf_counter()
wld = Arena(p1, p2, game).playGames(games)
total = time.perf_counter() - t0

board = game.getInitBoard()
g = pnet._graph1("both")
for _ in range(50):
    g.run(board)
n = 2000
t1 = time.perf_counter()
for _ in range(n):
    g.run(board)
replay_us = (time.perf_counter() - t1) / n * 1e6
out = {"games": games, "wld": list(wld), "seconds": round(total, 3),
       "games_per_s": round(games / total, 3), "net_calls": stat["calls"],
       "net_s": round(stat["net_s"], 3), "net_frac": round(stat["net_s"] / total, 3),
       "us_per_net_call": round(stat["net_s"] / max(1, stat["calls"]) * 1e6, 1),
       "host_us_per_call": round((total - stat["net_s"]) / max(1, stat["calls"]) * 1e6, 1),
       "graph_run_us_tight_loop": round(replay_us, 1)}
print(json.dumps(out), flush=True)

"""Arena gating speed (Coach.py:137-145): Connect4 7x7 GNN players, numMCTSSims 100, on the GPU;
the reference-shaped Python MCTS players vs the native-engine players (same games)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from types import SimpleNamespace  # noqa: E402

from Arena import Arena  # noqa: E402
from MCTS import MCTS  # noqa: E402
from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402
from mcts_native import ArenaPlayer  # noqa: E402

games = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 4
args = SimpleNamespace(numMCTSSims=100, cpuct=1.0, use_gnn=True, dropout=0.3, gnn_layers=2)
game = Connect4Game(7)
torch.manual_seed(0)
pnet, nnet = Connect4GNNWrapper(game, args), Connect4GNNWrapper(game, args)
out = {}
# warm-up leg first (allocations, graph capture), then each leg timed
legs = ["warmup", "native_speculative", "native_batch1", "native_speculative2", "native_batch1_2"] + (["python"] if "--python" in sys.argv else [])
for leg in legs:
    np.random.seed(7)
    native = leg != "python"
    if native:
        pf = "speculative" in leg or leg == "warmup"
        p1 = ArenaPlayer(game, pnet, args, prefetch=pf)
        p2 = ArenaPlayer(game, nnet, args, prefetch=pf)
    else:
        pm, nm = MCTS(game, pnet, args), MCTS(game, nnet, args)
        p1 = lambda x: np.argmax(pm.getActionProb(x, temp=0))  # noqa: E731
        p2 = lambda x: np.argmax(nm.getActionProb(x, temp=0))  # noqa: E731
    t0 = time.perf_counter()
    wld = Arena(p1, p2, game).playGames(games)
    dt = time.perf_counter() - t0
    out[leg] = {"wld": wld, "seconds": round(dt, 2), "games_per_s": round(games / dt, 3)}
    if native:
        out[leg].update(calls=p1.calls + p2.calls, hits=p1.hits + p2.hits)
    print(json.dumps(out), flush=True)

# per-call latency of the network entry points the arena uses (board in, numpy out)
z = np.zeros((8, 7, 7), np.int64)
lat = {}
for B in (1, 2, 8):
    for _ in range(50):
        pnet.predict_both(z[:B])
    t0 = time.perf_counter()
    for _ in range(500):
        pnet.predict_both(z[:B])
    lat["predict_both_B%d_us" % B] = round((time.perf_counter() - t0) / 500 * 1e6, 2)
out["latency"] = lat
print(json.dumps(out), flush=True)

"""Batch-1 hipGraph replay anatomy (run under rocprofv3 --kernel-trace --memory-copy-trace):
200 replays of the predict_both graph, then 200 eager predict_both calls with graphs disabled."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from types import SimpleNamespace  # noqa: E402

from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402

args = SimpleNamespace(numMCTSSims=100, cpuct=1.0, use_gnn=True, dropout=0.3, gnn_layers=2)
game = Connect4Game(7)
net = Connect4GNNWrapper(game, args)
board = game.getInitBoard()
g = net._graph1("both")
for _ in range(50):
    g.run(board)
t0 = time.perf_counter()
for _ in range(200):
    g.run(board)
print("graph us", (time.perf_counter() - t0) / 200 * 1e6, flush=True)
os.environ["AZ_NO_GRAPH"] = "1"
for _ in range(20):
    net.predict_both([board])
t0 = time.perf_counter()
for _ in range(200):
    net.predict_both([board])
print("eager us", (time.perf_counter() - t0) / 200 * 1e6, flush=True)

"""Host-side costs of one batch-1 evaluation: graph replay launch, stream synchronise on an idle
stream, synchronise after a replay, and the numpy staging writes/reads.  One JSON line."""
import json
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
s = torch.cuda.current_stream()
for _ in range(50):
    g.run(board)
out = {}


def t(name, fn, n=1000):
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    out[name] = round((time.perf_counter() - t0) / n * 1e6, 2)


t("run_us", lambda: g.run(board))
t("idle_sync_us", s.synchronize)
print(json.dumps({"batch1_class": type(g).__name__, "run_us": out["run_us"]}), flush=True)
from azhip.wrappers import _Batch1Graph  # noqa: E402
g = _Batch1Graph(net, "both")
for _ in range(50):
    g.run(board)
t("graph_run_us", lambda: g.run(board))
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100):
    g.graph.replay()
out["replay_launch_us"] = round((time.perf_counter() - t0) / 100 * 1e6, 2)
torch.cuda.synchronize()


def rs():
    g.graph.replay()
    s.synchronize()


t("replay_sync_us", rs)
t("stage_in_us", lambda: g.h_in.numpy().__setitem__(0, board))
t("stage_out_us", lambda: g.h_out.numpy()[0].copy())
e = torch.cuda.Event()


def rq():
    g.graph.replay()
    e.record()
    while not e.query():
        pass


t("replay_eventspin_us", rq)
print(json.dumps(out), flush=True)

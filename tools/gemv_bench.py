"""Batch-1 latency: az_gemm_f32 at M=1..8 on the output_transform shape (N=K=3136) and the
predict_both hipGraph replay (H2D, trunk, two GEMVs, heads, D2H, sync).  One JSON line."""
import json
import os
os.environ.setdefault("AZ_TUNING_LIB", "1")   # A/B switches live in the tuning build
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from types import SimpleNamespace  # noqa: E402

from azhip import ops  # noqa: E402
from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402

F = 3136
w = torch.randn(F, F, device="cuda") / F ** 0.5
b = torch.randn(F, device="cuda")
out = {"variant": {k: os.environ[k] for k in ("AZ_GEMV_CHUNKED", "AZ_GEMV_R") if k in os.environ}}
for M in (1, 2, 4, 8):
    x = torch.randn(M, F, device="cuda")
    y = torch.empty(M, F, device="cuda")
    for _ in range(20):
        ops.linear(x, w, b, act=ops.ACT_RELU, out=y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        ops.linear(x, w, b, act=ops.ACT_RELU, out=y)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 200
    out[f"M{M}_us"] = round(us, 2)
    out[f"M{M}_GBps"] = round(F * F * 4 / us / 1e3, 1)
args = SimpleNamespace(numMCTSSims=100, cpuct=1.0, use_gnn=True, dropout=0.3, gnn_layers=2)
game = Connect4Game(7)
net = Connect4GNNWrapper(game, args)
board = game.getInitBoard()
g = net._graph1("both")
for _ in range(50):
    g.run(board)
t0 = time.perf_counter()
for _ in range(2000):
    g.run(board)
out["graph_both_us"] = round((time.perf_counter() - t0) / 2000 * 1e6, 1)
print(json.dumps(out), flush=True)

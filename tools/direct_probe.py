"""_Batch1Direct anatomy: host time of the az_c4_eval_fwd call (4 launches), of the stream
synchronise that follows, and the GPU time of the launch chain (events).  One JSON line."""
import ctypes
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
d = net._graph1("both")
s = torch.cuda.current_stream()
sp = ctypes.c_void_p(s.cuda_stream)
for _ in range(50):
    d.run(board)
n = 2000
tc = ts = 0.0
for _ in range(n):
    t0 = time.perf_counter()
    d.fn(*d.args, sp)
    t1 = time.perf_counter()
    s.synchronize()
    t2 = time.perf_counter()
    tc += t1 - t0
    ts += t2 - t1
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
gpu = 0.0
for _ in range(200):
    e0.record()
    d.fn(*d.args, sp)
    e1.record()
    e1.synchronize()
    gpu += e0.elapsed_time(e1) * 1e3
# back-to-back chains (no sync between): throughput limit of host launch vs GPU
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(500):
    d.fn(*d.args, sp)
torch.cuda.synchronize()
b2b = (time.perf_counter() - t0) / 500 * 1e6
print(json.dumps({"call_us": round(tc / n * 1e6, 2), "sync_us": round(ts / n * 1e6, 2),
                  "gpu_chain_us": round(gpu / 200, 2), "back_to_back_us": round(b2b, 2)}),
      flush=True)

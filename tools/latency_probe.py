"""Per-call latency of the as-called network entry points on the GPU (arena / sequential MCTS):
predict_both on B = 1..8 Connect4 7x7 boards (one az_c4_eval_fwd call).  Run under
`rocprofv3 --kernel-trace --stats` to split a call into kernel time and host/launch time."""
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
game = Connect4Game(7)
torch.manual_seed(0)
w = Connect4GNNWrapper(game, SimpleNamespace(dropout=0.3, gnn_layers=2))
z = np.zeros((8, 7, 7), np.int64)
lat = {}
for B in (1, 2, 4, 8):
    for _ in range(50):
        w.predict_both(z[:B])
    t0 = time.perf_counter()
    for _ in range(n):
        w.predict_both(z[:B])
    lat["predict_both_B%d_us" % B] = round((time.perf_counter() - t0) / n * 1e6, 2)
for name, f in (("predict", w.predict), ("predict_with_gnn", w.predict_with_gnn)):
    for _ in range(50):
        f(z[0])
    t0 = time.perf_counter()
    for _ in range(n):
        f(z[0])
    lat[name + "_us"] = round((time.perf_counter() - t0) / n * 1e6, 2)
print(json.dumps(lat), flush=True)

"""Config 5: PolicyValueGNN(64, 2 layers) forward over 32x32 grid graphs
(per-destination generalisation of gnn_utils.py:34-117) on one GPU: time per forward and the
per-kernel split (run under rocprofv3 for the latter).   python tools/grid_forward.py [graphs]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
import bench  # noqa: E402
from azhip import ops  # noqa: E402
from azhip.nets import PolicyValueGNN  # noqa: E402
from azhip.weights import gnn_spec, synthetic_state_dict  # noqa: E402

graphs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
g = bench._grid_graph(ops, dev, graphs)
net = PolicyValueGNN(64, 2, device=dev, init=synthetic_state_dict(gnn_spec(64, 2), 3)).eval()
x = torch.rand((g.V, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 2 - 1
for _ in range(3):
    y = net.forward_graph(x, g)
torch.cuda.synchronize()
reps = 10
t0 = time.perf_counter()
for _ in range(reps):
    y = net.forward_graph(x, g)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
# 73,728 FLOP/node/layer + 640 FLOP/edge/layer + 16,384 FLOP/node output_transform
flop = 2 * (73728 * g.V + 640 * g.E) + 16384 * g.V
print(json.dumps({"graphs": graphs, "V": g.V, "E": g.E, "ms_per_forward": round(dt * 1e3, 3),
                  "node_updates_per_s": round(2 * g.V / dt, 1),
                  "gflop_per_forward": round(flop / 1e9, 2),
                  "tflops": round(flop / dt / 1e12, 2)}))

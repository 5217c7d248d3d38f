"""M=1 GEMV GPU time vs weight size, 50 launches per hipGraph (launch cost amortised): the
bandwidth the batch-1 path gets from L2 / Infinity Cache / HBM.  One JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402

out = {}
R = 50
for N, K in ((1024, 1024), (2048, 2048), (3136, 3136), (6272, 3136), (12544, 3136),
             (25088, 3136)):
    w = torch.randn(N, K, device="cuda")
    x = torch.randn(1, K, device="cuda")
    y = torch.empty(1, N, device="cuda")
    ops.linear(x, w, None, out=y)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(R):
            ops.linear(x, w, None, out=y)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (4 * R)
    out[f"{N}x{K}"] = {"MB": round(N * K * 4 / 1e6, 1), "us": round(us, 2),
                       "GBps": round(N * K * 4 / us / 1e3, 1)}
print(json.dumps(out), flush=True)

"""c4_trunk GPU time at B = 1 / 512 / 4096 (50 launches in one hipGraph, event-timed).
One JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402
from azhip.weights import connect4_net_spec, synthetic_state_dict  # noqa: E402

W = {k: torch.from_numpy(v).cuda() for k, v in synthetic_state_dict(connect4_net_spec(7), 1).items()}
out = {}
R = 50
for B in (1, 512, 4096):
    boards = torch.from_numpy(np.random.default_rng(0).integers(-1, 2, (B, 7, 7)).astype(np.int8)).cuda()
    feat = torch.empty((B, 3136), device="cuda")
    ops.c4_trunk(boards, W, out=feat)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(R):
            ops.c4_trunk(boards, W, out=feat)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    out[f"B{B}_us"] = round(e0.elapsed_time(e1) * 1e3 / (4 * R), 2)
print(json.dumps(out), flush=True)

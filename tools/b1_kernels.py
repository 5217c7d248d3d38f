"""GPU-side time of each batch-1 kernel: 50 back-to-back launches captured in one hipGraph and
replayed (host launch cost amortised), timed with events.  One JSON line (us per launch)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from types import SimpleNamespace  # noqa: E402

from azhip import ops  # noqa: E402
from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402

args = SimpleNamespace(numMCTSSims=100, cpuct=1.0, use_gnn=True, dropout=0.3, gnn_layers=2)
net = Connect4GNNWrapper(Connect4Game(7), args)
net.nnet.eval()
net.gnn.eval()
W, G = net.nnet.params, net.gnn.params
b = torch.zeros((1, 7, 7), dtype=torch.int8, device="cuda")
hb = ops.HostBuffer(4096)
bh = hb.view(0, torch.int8, (1, 7, 7))
oh = hb.view(256, torch.float32, (1, 18))
f = ops.c4_trunk(b, W)
x = torch.randn(1, 3136, device="cuda")
h = torch.empty(1, 3136, device="cuda")
ws = torch.empty(16 << 20, dtype=torch.uint8, device="cuda")
R = 50


def timed(name, fn):
    with ops.pinned_workspace(torch.device("cuda", 0), ws):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(R):
                fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    out[name] = round(e0.elapsed_time(e1) * 1e3 / (5 * R), 2)


out = {}
timed("trunk_dev", lambda: ops.c4_trunk(b, W, out=f))
timed("trunk_hostboard", lambda: ops.c4_trunk(bh, W, out=f))
timed("trunk_heads_hostio", lambda: net.nnet.features_heads(bh, pi=oh[:, :8], v=oh[:, 8]))
timed("trunk_heads_dev", lambda: net.nnet.features_heads(b))
timed("gemv_3136", lambda: ops.linear(x, G["output_transform.0.weight"],
                                      G["output_transform.0.bias"], act=ops.ACT_RELU, out=h))
timed("heads_rows_dev", lambda: net.nnet.heads(x))
timed("heads_rows_hostout", lambda: net.nnet.heads(x, pi=oh[:, :8], v=oh[:, 8]))
timed("gnn_tail_dev", lambda: ops.transform_heads(
    f, G["output_transform.0.weight"], G["output_transform.0.bias"],
    G["output_transform.2.weight"], G["output_transform.2.bias"], W["fc_policy.weight"],
    W["fc_policy.bias"], W["fc_value.weight"], W["fc_value.bias"]))
timed("empty_fill", lambda: h.fill_(0))
print(json.dumps(out), flush=True)

"""Eager vs hipGraph-replayed Connect4 GNN eval step (trunk -> output_transform -> heads),
B = 512: does capturing the 6 launches in one graph shorten the step?"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402
from azhip.nets import C4Evaluator  # noqa: E402
from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict  # noqa: E402

B, F = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 3136
ev = C4Evaluator(synthetic_state_dict(connect4_net_spec(7), 1),
                 synthetic_state_dict(gnn_spec(F, 2), 2), device="cuda")
rng = np.random.default_rng(1)
boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)).cuda()
Wn, Gn = ev.nnet.params, ev.gnn.params
feat = torch.empty((B, F), device="cuda")
h, y = torch.empty((B, F), device="cuda"), torch.empty((B, F), device="cuda")
logp, pi, v = (torch.empty((B, 8), device="cuda"), torch.empty((B, 8), device="cuda"),
               torch.empty((B,), device="cuda"))


def step():
    ops.c4_trunk(boards, Wn, out=feat)
    ops.transform_heads(feat, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                        Gn["output_transform.2.weight"], Gn["output_transform.2.bias"],
                        Wn["fc_policy.weight"], Wn["fc_policy.bias"], Wn["fc_value.weight"],
                        Wn["fc_value.bias"], hidden=h, y=y, logp=logp, pi=pi, v=v)


for _ in range(10):
    step()
torch.cuda.synchronize()
ref = (pi.clone(), v.clone())
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
pi.zero_(); v.zero_()
g.replay()
torch.cuda.synchronize()
assert torch.equal(pi, ref[0]) and torch.equal(v, ref[1]), "graph replay differs"
evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def step_ev():
    ops.c4_trunk(boards, Wn, out=feat)
    evs[0].record()
    ops.linear(feat, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
               act=ops.ACT_RELU, out=h)
    evs[1].record()
    ops.linear_heads(h, Gn["output_transform.2.weight"], Gn["output_transform.2.bias"],
                     Wn["fc_policy.weight"], Wn["fc_policy.bias"], Wn["fc_value.weight"],
                     Wn["fc_value.bias"], y=y, logp=logp, pi=pi, v=v)


def step_split():
    ops.c4_trunk(boards, Wn, out=feat)
    ops.linear(feat, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
               act=ops.ACT_RELU, out=h)
    ops.linear_heads(h, Gn["output_transform.2.weight"], Gn["output_transform.2.bias"],
                     Wn["fc_policy.weight"], Wn["fc_policy.bias"], Wn["fc_value.weight"],
                     Wn["fc_value.bias"], y=y, logp=logp, pi=pi, v=v)


for name, fn in (("eager", step), ("graph", g.replay), ("split", step_split),
                 ("split+2ev", step_ev), ("eager", step), ("graph", g.replay),
                 ("split", step_split), ("split+2ev", step_ev)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    print(f"{name}: {us:.1f} us/step  {B / us * 1e6:.0f} boards/s", flush=True)

"""Batched predict_with_gnn step (bench.py's headline) as ONE az_c4_eval_fwd call with the
pre-split A hand-offs (ops.c4_gnn_eval) vs the unfused calls (trunk, then each GEMM splitting its
own A), alternated in one process: HIP-event time per step.
    python tools/presplit_probe.py [B ...]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "alphazero-gnn_amd"))
from azhip import ops  # noqa: E402
from azhip.nets import C4Evaluator  # noqa: E402
from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict  # noqa: E402

ev = C4Evaluator(synthetic_state_dict(connect4_net_spec(7), 1),
                 synthetic_state_dict(gnn_spec(3136, 2), 2), device=torch.device("cuda"))
Wn, Gn = ev.nnet.params, ev.gnn.params
for B in [int(b) for b in (sys.argv[1:] or ["512"])]:
    boards = torch.from_numpy(np.random.default_rng(B).integers(-1, 2, size=(B, 7, 7))
                              .astype(np.int8)).cuda()
    bufs = [torch.empty((B, 3136), device="cuda") for _ in range(3)]

    def fused():
        ops.c4_gnn_eval(boards, Wn, Gn, feat=bufs[0], hidden=bufs[1], y=bufs[2])

    def unfused():
        f = ops.c4_trunk(boards, Wn, out=bufs[0])
        ops.linear(f, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                   act=ops.ACT_RELU, out=bufs[1])
        ops.linear_heads(bufs[1], Gn["output_transform.2.weight"], Gn["output_transform.2.bias"],
                         Wn["fc_policy.weight"], Wn["fc_policy.bias"], Wn["fc_value.weight"],
                         Wn["fc_value.bias"], y=bufs[2])

    res = {}
    for _ in range(400):
        fused()
    for rep in range(3):
        for name, fn in (("fused", fused), ("unfused", unfused)):
            for _ in range(50):
                fn()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record()
            for _ in range(200):
                fn()
            e[1].record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(round(e[0].elapsed_time(e[1]) / 200 * 1e3, 2))
    print(json.dumps({"B": B, "us_per_step": res}), flush=True)

"""Probe: the Connect4 trunk (az_c4_trunk_fwd via c4_trunk_launch) at each B with registered
weights -- HIP-event time per call; AZ_TUNING_LIB=1 AZ_TRUNK_NO_W2F=1 stages conv2 through LDS
instead of the fragment-ordered copy (A/B); AZ_TUNING_LIB=1 AZ_TRUNK_NB=<n> forces n boards per
block (the rounds model's t(NB) sweep).  python tools/trunk_w2f_probe.py [B[,B...]] [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))


def main():
    import torch
    from azhip import ops
    from azhip.nets import C4Evaluator
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "512").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ev = C4Evaluator(synthetic_state_dict(connect4_net_spec(7), 1),
                     synthetic_state_dict(gnn_spec(3136, 2), 2), device=torch.device("cuda"))
    for B in Bs:
        one(torch, ops, ev, B, reps)


def one(torch, ops, ev, B, reps):
    b = torch.from_numpy(np.random.default_rng(0).integers(-1, 2, (B, 7, 7)).astype(np.int8)).cuda()
    f = ops.c4_trunk(b, ev.nnet.params)
    for _ in range(50):
        ops.c4_trunk(b, ev.nnet.params, out=f)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        ops.c4_trunk(b, ev.nnet.params, out=f)
    e[1].record()
    torch.cuda.synchronize()
    print(f"B={B} trunk_us={e[0].elapsed_time(e[1]) / reps * 1e3:.2f} "
          f"w2f={'off' if os.environ.get('AZ_TRUNK_NO_W2F') else 'on'} "
          f"nb={os.environ.get('AZ_TRUNK_NB', 'model')} "
          f"sum={float(f.double().sum()):.6f}", flush=True)


if __name__ == "__main__":
    main()

"""The Connect4 trunk's three launch forms at self-play batch sizes, back to back on one stream,
for a kernel trace (rocprofv3 --kernel-trace --stats): c4_trunk_kernel (ops.c4_trunk, features
only), c4_trunk_split_a_kernel<NB, false> (ops.c4_gnn_eval: + output_transform.0's pre-split A)
and c4_trunk_split_a_kernel<NB, true> (predict_both: + the standard heads from the LDS rows).
    python tools/trunk_variants_probe.py [B,B,...] [reps]"""
import os
import sys
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))


def main():
    import torch
    from azhip import ops
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1576,3150").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    w = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(numMCTSSims=100, cpuct=1.0,
                                                            use_gnn=True, dropout=0.3,
                                                            gnn_layers=2))
    w.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synthetic_state_dict(connect4_net_spec(7), 1).items()})
    w.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in
                           synthetic_state_dict(gnn_spec(3136, 2), 2).items()})
    Wn, Gn = w.nnet.params, w.gnn.params
    for B in Bs:
        b = np.random.default_rng(B).integers(-1, 2, size=(B, 7, 7)).astype(np.int8)
        bd = torch.from_numpy(b).cuda()
        feat = torch.empty((B, 3136), device="cuda")
        hidden = torch.empty((B, 3136), device="cuda")
        for _ in range(3):
            ops.c4_trunk(bd, Wn)
            ops.c4_gnn_eval(bd, Wn, Gn, feat=feat, hidden=hidden)
            w.predict_both_async(b).result()
        torch.cuda.synchronize()
        for _ in range(reps):
            ops.c4_trunk(bd, Wn)
        for _ in range(reps):
            ops.c4_gnn_eval(bd, Wn, Gn, feat=feat, hidden=hidden)
        for _ in range(reps):
            w.predict_both_async(b).result()
        torch.cuda.synchronize()
        print(f"B={B} done", flush=True)


if __name__ == "__main__":
    main()

"""Probe: rows of the async lock-step path (_DirectBatch, az_c4_eval_fwd with a cap-1024
descriptor) vs the batch-1 path for n = 1..16 boards, with one and with two batches in flight.
Prints the max |diff| per case (GPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from types import SimpleNamespace
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    W = synthetic_state_dict(connect4_net_spec(7), 1)
    G = synthetic_state_dict(gnn_spec(3136, 2), 2)
    net = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(dropout=0.3, gnn_layers=2))
    net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in G.items()})
    rng = np.random.default_rng(0)
    boards = rng.integers(-1, 2, size=(64, 7, 7)).astype(np.int8)
    one = [net.predict_both(boards[i:i + 1].astype(np.int64)) for i in range(64)]

    def diff(out, idx):
        d = 0.0
        for r, i in enumerate(idx):
            for k in range(4):
                d = max(d, float(np.abs(np.asarray(out[k][r]) - np.asarray(one[i][k][0])).max()))
        return d

    for n in (1, 2, 3, 5, 8, 9, 16, 33):
        idx = list(range(n))
        out = net.predict_both_async(boards[idx]).result()
        d1 = diff(out, idx)
        idx2 = list(range(20, 20 + n))
        pa = net.predict_both_async(boards[idx])
        pb = net.predict_both_async(boards[idx2])
        oa, ob = pa.result(), pb.result()
        d2 = max(diff(oa, idx), diff(ob, idx2))
        ob2 = pb.result() if False else None
        # reversed read order
        pa = net.predict_both_async(boards[idx])
        pb = net.predict_both_async(boards[idx2])
        ob, oa = pb.result(), pa.result()
        d3 = max(diff(oa, idx), diff(ob, idx2))
        sync = net.predict_both(boards[idx].astype(np.int64))
        d4 = diff(sync, idx)
        print(f"n={n:3d} async-one {d1:.3g}  two-in-flight {d2:.3g}  reversed {d3:.3g}  "
              f"sync predict_both {d4:.3g}", flush=True)


if __name__ == "__main__":
    main()

"""The batch-1..8 evaluator call (the arena's speculative leaf batches) with and without the
one-launch leaf kernel: median us per call for each row count.   python tools/leaf_rows_probe.py"""
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))


def main():
    import torch
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    from azhip.wrappers import _Batch1Direct
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    w = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(numMCTSSims=100, cpuct=1.0,
                                                            use_gnn=True, dropout=0.3,
                                                            gnn_layers=2))
    w.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synthetic_state_dict(connect4_net_spec(7), 1).items()})
    w.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in
                           synthetic_state_dict(gnn_spec(3136, 2), 2).items()})
    w.nnet.eval()
    w.gnn.eval()
    fused, plain = _Batch1Direct(w, "both", cap=8), _Batch1Direct(w, "both", cap=8)
    plain.desc.sync = plain.desc.err = None
    plain.err_np = None
    b = np.random.default_rng(0).integers(-1, 2, size=(8, 7, 7)).astype(np.int8)
    out = {}
    for n in range(1, 9):
        row = {}
        for name, d in (("fused", fused), ("four_launches", plain)):
            for _ in range(50):
                d.run_rows(b[:n])
            ts = []
            for _ in range(1500):
                t = time.perf_counter()
                d.run_rows(b[:n])
                ts.append(time.perf_counter() - t)
            row[name] = round(float(np.median(ts)) * 1e6, 2)
        out[n] = row
        print(json.dumps({"rows": n, **row}), flush=True)


if __name__ == "__main__":
    main()

"""One self-play round's GPU work in isolation: predict_both_async on M random boards (the lock-step
lane's batch), back to back on one stream; run under rocprofv3 --kernel-trace --stats for the
per-kernel split at self-play shapes.   python tools/sp_round_probe.py [M] [reps]"""
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
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 1576
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    w = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(numMCTSSims=100, cpuct=1.0,
                                                            use_gnn=True, dropout=0.3,
                                                            gnn_layers=2))
    w.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synthetic_state_dict(connect4_net_spec(7), 1).items()})
    w.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in
                           synthetic_state_dict(gnn_spec(3136, 2), 2).items()})
    b = np.random.default_rng(0).integers(-1, 2, size=(M, 7, 7)).astype(np.int8)
    for _ in range(3):
        w.predict_both_async(b).result()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        w.predict_both_async(b).result()
    dt = (time.perf_counter() - t) / reps
    print(f"M={M} us_per_round={dt * 1e6:.1f}", flush=True)


if __name__ == "__main__":
    main()

"""Probe: what data-parallel training saves per GNN step.

On one GPU, time the GNN training step (Connect4GNN.py:160-197: star of 64 rows, 2 layers,
output_transform, heads, loss, backward, Adam over 119.6 M parameters):
  replicas -- train.gnn_step, the whole batch (what every rank runs under "replicas");
  dp P     -- train.gnn_step_dp as rank 0 of P ranks with the collectives stubbed out (the
              gathered features are this rank's rows zero-padded; broadcast / all_reduce are
              no-ops): the compute one rank does per step under "allreduce", for P = 2, 4, 8.
The difference is the compute DP removes per step; the row0 form adds an all_reduce of 78.7 MB
(output_transform's gradient) + a 12.5 KB broadcast + an 800 KB all_gather, the flat form an
all_reduce of 478.6 MB.  Prints one JSON line per case.
  python tools/dp_step_probe.py [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))


def main():
    import torch
    from types import SimpleNamespace
    from azhip import dist as D
    from azhip import train as T
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    W = synthetic_state_dict(connect4_net_spec(7), 1)
    G = synthetic_state_dict(gnn_spec(3136, 2), 2)
    args = SimpleNamespace(lr=0.001, dropout=0.3, epochs=1, batch_size=64, gnn_layers=2,
                           use_gnn=True)
    w = Connect4GNNWrapper(Connect4Game(7), args)
    w.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    w.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in G.items()})
    w.nnet.train()
    w.gnn.train()
    rng = np.random.default_rng(0)
    B = 64
    dev = w.device
    boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)).to(dev)
    tpi = torch.from_numpy(rng.dirichlet(np.ones(8), B).astype(np.float32)).to(dev)
    tv = torch.from_numpy(rng.uniform(-1, 1, B).astype(np.float32)).to(dev)
    w.gnn.params.reset_adam()

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    rep_ms = timed(lambda: T.gnn_step(w.nnet, w.gnn, boards, tpi, tv, 1e-9, seed=1))
    print(json.dumps({"case": "replicas", "ms_per_gnn_step": round(rep_ms, 3)}), flush=True)
    orig = (D.world_rank, D.gather_rows, D.allreduce_sum_, D.broadcast_)
    for P in (2, 4, 8):
        def gather(own, n, world, rank):
            full = torch.zeros((n, own.shape[1]), dtype=own.dtype, device=own.device)
            r0, r1 = D.row_shard(n, world, rank)
            full[r0:r1] = own
            return full
        D.world_rank = lambda P=P: (P, 0)
        D.gather_rows, D.allreduce_sum_, D.broadcast_ = gather, (lambda t: t), (lambda t, src=0: t)
        try:
            for sync in ("row0", "flat"):
                ms = timed(lambda: T.gnn_step_dp(w.nnet, w.gnn, boards, tpi, tv, 1e-9, seed=1,
                                                 grad_sync=sync))
                print(json.dumps({"case": f"dp{P}", "grad_sync": sync,
                                  "ms_per_gnn_step_rank0_compute": round(ms, 3),
                                  "saved_ms_vs_replicas": round(rep_ms - ms, 3),
                                  "allreduce_bytes": 78.7e6 if sync == "row0" else 478.6e6}),
                      flush=True)
        finally:
            D.world_rank, D.gather_rows, D.allreduce_sum_, D.broadcast_ = orig


if __name__ == "__main__":
    main()

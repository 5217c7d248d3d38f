"""Host side of the batch-1 leaf call (the arena's predict_both): where the microseconds between
the Python call and the result go.  Times, per call (median of N):
  full      net.predict_both(board) as MCTS / the arena call it
  run_rows  the evaluator alone (_Batch1Direct.run_rows)
  c+sync    the ctypes az_c4_eval_fwd call + stream synchronize only
  c+spin    the ctypes call, then an event polled by query() in a spin loop
  stream    torch.cuda.current_stream() alone
  sync_idle synchronize() of an idle stream
  python tools/b1_host_probe.py [calls]"""
import ctypes
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))


def med(f, n):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return round(float(np.median(ts)) * 1e6, 2)


def main():
    import torch
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    w = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(numMCTSSims=100, cpuct=1.0,
                                                            use_gnn=True, dropout=0.3,
                                                            gnn_layers=2))
    w.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synthetic_state_dict(connect4_net_spec(7), 1).items()})
    w.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in
                           synthetic_state_dict(gnn_spec(3136, 2), 2).items()})
    b = np.random.default_rng(0).integers(-1, 2, size=(1, 7, 7)).astype(np.int8)
    w.predict_both(b)
    d = w._g1["both"]
    s = torch.cuda.current_stream()
    ptr = ctypes.c_void_p(s.cuda_stream)
    ev = torch.cuda.Event()

    def csync():
        d.fn(*d.args, 1, *d.outs, ptr)
        s.synchronize()

    def cspin():
        d.fn(*d.args, 1, *d.outs, ptr)
        ev.record(s)
        while not ev.query():
            pass

    out = {"calls": n, "unit": "us per call (median)",
           "full": med(lambda: w.predict_both(b), n),
           "run_rows": med(lambda: d.run_rows(b), n),
           "c+sync": med(csync, n), "c+spin": med(cspin, n),
           "stream": med(lambda: torch.cuda.current_stream(), n),
           "sync_idle": med(lambda: s.synchronize(), n),
           "fused": bool(d.desc.sync)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

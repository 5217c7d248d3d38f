"""Where c4_leaf_kernel's time goes (tuning build, AZ_LEAF_TRACE): per event the earliest and
latest block stamp (100 MHz wall clock) relative to the first block's start, median over leaves.
  AZ_TUNING_LIB=1 AZ_LEAF_TRACE=1 python tools/leaf_probe.py [leaves]"""
import ctypes
import json
import os
import sys
from types import SimpleNamespace

import numpy as np

os.environ.setdefault("AZ_TUNING_LIB", "1")
os.environ.setdefault("AZ_LEAF_TRACE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))

EVENTS = ["start", "trunk", "g1_weights", "g1_go", "g1_done", "g2_weights", "g2_go", "g2_done",
          "chunk", "final", "std_heads"]


def main():
    import torch
    from azhip import _lib
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    from azhip.wrappers import _Batch1Direct
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    w = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(numMCTSSims=100, cpuct=1.0,
                                                            use_gnn=True, dropout=0.3,
                                                            gnn_layers=2))
    w.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synthetic_state_dict(connect4_net_spec(7), 1).items()})
    w.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in
                           synthetic_state_dict(gnn_spec(3136, 2), 2).items()})
    w.nnet.eval()
    w.gnn.eval()
    d = _Batch1Direct(w, "both", cap=8)
    L = _lib.lib()
    L.az_tuning_leaf_trace.restype = ctypes.c_int
    L.az_tuning_leaf_trace.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(0)
    out = np.zeros(2 * len(EVENTS), np.uint64)
    rows = []
    for i in range(n):
        b = rng.integers(-1, 2, size=(1, 7, 7)).astype(np.int8)
        d.run_rows(b)
        assert L.az_tuning_leaf_trace(out.ctypes.data) == len(EVENTS)
        t0 = int(out[0])
        rows.append([((int(out[2 * e]) - t0) / 100.0 if out[2 * e] != np.uint64(2 ** 64 - 1) else -1,
                      (int(out[2 * e + 1]) - t0) / 100.0 if out[2 * e + 1] else -1)
                     for e in range(len(EVENTS))])
    med = np.median(np.array(rows[5:]), axis=0)
    print(json.dumps({"leaves": n, "unit": "us after the first block started",
                      "events": {EVENTS[e]: {"first": round(float(med[e][0]), 2),
                                             "last": round(float(med[e][1]), 2)}
                                 for e in range(len(EVENTS))}}, indent=1))


if __name__ == "__main__":
    main()

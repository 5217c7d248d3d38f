"""Probe: host time of one predict_both_async launch (az_c4_eval_fwd's host side: argument
checks, plans, kernel launches) per batch size, GPU idle before each call.
    python tools/launch_host_probe.py [B,B,...]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    import bench
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    sa = bench.selfplay_args(100)
    net = Connect4GNNWrapper(Connect4Game(7), sa)
    net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in
                              synthetic_state_dict(connect4_net_spec(7), 1).items()})
    net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in
                             synthetic_state_dict(gnn_spec(3136, 2), 2).items()})
    s = torch.cuda.Stream()
    Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                           "300,400,700,1000,1300,1576,1800,2103,2400,3150,4096").split(",")]
    rng = np.random.default_rng(0)
    net.predict_both_async(rng.integers(-1, 2, size=(4096, 7, 7)).astype(np.int8), stream=s).result()
    for B in Bs:
        boards = rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)
        ts, tw = [], []
        for rep in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p = net.predict_both_async(boards[:B - rep], stream=s)   # a new M each call
            t1 = time.perf_counter()
            p.result()
            t2 = time.perf_counter()
            ts.append(t1 - t0)
            tw.append(t2 - t1)
        print(json.dumps({"B": B, "launch_ms": [round(t * 1e3, 3) for t in ts],
                          "wait_ms": round(float(np.median(tw)) * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()

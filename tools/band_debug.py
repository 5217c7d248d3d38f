"""Band-kernel bisection (GPU): the eval-mode band layer vs the training path under weight sets
that switch phases off one at a time, printing the error per case.

    python tools/band_debug.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "alphazero-gnn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from azhip import ops  # noqa: E402


def band_graph(V, maxdeg, R, seed):
    rng = np.random.default_rng(seed)
    rowptr, col = [0], []
    for d in range(V):
        k = int(rng.integers(1, maxdeg + 1))
        lo, hi = max(0, d - R), min(V - 1, d + R)
        src = np.sort(rng.choice(np.arange(lo, hi + 1), size=k, replace=False))
        col += src.tolist()
        rowptr.append(len(col))
    return np.array(rowptr), np.array(col)


def main():
    dev = torch.device("cuda:0")
    V = 256
    rowptr, col = band_graph(V, 4, 32, 1)
    g = ops.DeviceGraph(rowptr, col)
    rng = np.random.default_rng(0)
    x0 = (rng.random((V, 64), dtype=np.float32) * 2 - 1)
    x = torch.from_numpy(x0).to(dev)

    def rnd(*s, sc=0.1):
        return torch.from_numpy((rng.standard_normal(s) * sc).astype(np.float32)).to(dev)

    base = {"attention.0.weight": rnd(128, 128), "attention.0.bias": rnd(128),
            "attention.2.weight": rnd(1, 128), "attention.2.bias": rnd(1),
            "gate.0.weight": rnd(64, 128), "gate.0.bias": rnd(64),
            "update_net.0.weight": rnd(64, 128), "update_net.0.bias": rnd(64),
            "update_net.2.weight": rnd(64, 64), "update_net.2.bias": rnd(64)}
    eye = torch.eye(64, device=dev)
    z64 = torch.zeros(64, 64, device=dev)
    cases = {
        "random": {},
        "gate0": {"gate.0.weight": torch.zeros(64, 128, device=dev),
                  "gate.0.bias": torch.full((64,), -40.0, device=dev)},
        "x_half": {"gate.0.weight": torch.zeros(64, 128, device=dev),
                   "gate.0.bias": torch.full((64,), 40.0, device=dev),
                   "update_net.0.weight": torch.cat([eye, z64], 1),
                   "update_net.0.bias": torch.zeros(64, device=dev),
                   "update_net.2.weight": eye.clone(),
                   "update_net.2.bias": torch.zeros(64, device=dev)},
        "agg_half": {"gate.0.weight": torch.zeros(64, 128, device=dev),
                     "gate.0.bias": torch.full((64,), 40.0, device=dev),
                     "update_net.0.weight": torch.cat([z64, eye], 1),
                     "update_net.0.bias": torch.zeros(64, device=dev),
                     "update_net.2.weight": eye.clone(),
                     "update_net.2.bias": torch.zeros(64, device=dev)},
        "agg_half_att0": {"attention.0.weight": torch.zeros(128, 128, device=dev),
                          "gate.0.weight": torch.zeros(64, 128, device=dev),
                          "gate.0.bias": torch.full((64,), 40.0, device=dev),
                          "update_net.0.weight": torch.cat([z64, eye], 1),
                          "update_net.0.bias": torch.zeros(64, device=dev),
                          "update_net.2.weight": eye.clone(),
                          "update_net.2.bias": torch.zeros(64, device=dev)},
        "u2_only": {"gate.0.weight": torch.zeros(64, 128, device=dev),
                    "gate.0.bias": torch.full((64,), 40.0, device=dev),
                    "update_net.0.weight": torch.zeros(64, 128, device=dev),
                    "update_net.0.bias": torch.ones(64, device=dev),
                    "update_net.2.weight": eye.clone(),
                    "update_net.2.bias": torch.zeros(64, device=dev)},
    }
    for name, over in cases.items():
        W = dict(base)
        W.update(over)
        a, _ = ops.gnn_layer(g, x, W, save=True)
        b, _ = ops.gnn_layer(g, x, W, save=False)
        a, b = a.cpu().numpy(), b.cpu().numpy()
        err = np.abs(a - b)
        rows = np.argwhere(err.max(1) > 1e-4).ravel()
        cols = np.argwhere(err.max(0) > 1e-4).ravel()
        print(f"{name:14s} max {err.max():.3e}  bad rows {len(rows)} {rows[:8].tolist()}  "
              f"bad cols {len(cols)} {cols[:8].tolist()}")
        if len(rows):
            r = rows[0]
            print("   train", np.round(a[r, :8], 4).tolist())
            print("   band ", np.round(b[r, :8], 4).tolist())
            print("   x    ", np.round(x0[r, :8], 4).tolist())


if __name__ == "__main__":
    main()

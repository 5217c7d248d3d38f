"""Diagnose the band kernel vs the training path on rows of very different magnitudes."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from azhip import ops  # noqa: E402
from test_gpu_kernels import _synth, _band_graph  # noqa: E402


def main():
    _, G, _ = _synth()
    V = 3000
    rowptr, col = _band_graph(V, 4, 32, seed=77, p_empty=0.05)
    g = ops.DeviceGraph(rowptr, col)
    rng = np.random.default_rng(78)
    x0 = (rng.random((V, 64), dtype=np.float32) * 2 - 1)
    mag = rng.uniform(-15, 15, (V, 1))
    x0 *= (10.0 ** mag).astype(np.float32)
    x0[rng.random(V) < 0.05] = 0.0
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    Gd = {k: cu(v) for k, v in G.items()}
    x = cu(x0)
    Wl = {k[len("layers.1."):]: v for k, v in Gd.items() if k.startswith("layers.1.")}
    a, _ = ops.gnn_layer(g, x, Wl, save=True)
    b, _ = ops.gnn_layer(g, x, Wl, save=False)
    a, b = a.cpu().numpy().astype(np.float64), b.cpu().numpy().astype(np.float64)
    scale = np.maximum(np.abs(a).max(1), np.abs(x0).max(1))
    err = np.abs(b - a).max(1) / np.maximum(scale, 1e-30)
    order = np.argsort(-err)[:8]
    print("rows over 2e-5:", int((err > 2e-5).sum()), "of", V)
    for r in order:
        srcs = col[rowptr[r]:rowptr[r + 1]]
        print(f"row {r} err {err[r]:.3g} |x| {np.abs(x0[r]).max():.3g} |a| {np.abs(a[r]).max():.3g} "
              f"|b| {np.abs(b[r]).max():.3g} deg {len(srcs)} src|x| "
              f"{[float('%.2g' % np.abs(x0[s]).max()) for s in srcs]} tile {r // 64} pos {r % 64}")
        j = int(np.argmax(np.abs(b[r] - a[r])))
        print(f"    col {j}: a {a[r, j]:.6g} b {b[r, j]:.6g}")


if __name__ == "__main__":
    main()

"""Per-phase timeline of gnn_layer_band_kernel (tuning build, AZ_BAND_ABL=256: wall-clock stamps
of block 0's waves 0 and 4 at every phase boundary of its tiles).  Prints the median duration of
each stage over the block's tiles, in microseconds (100 MHz clock).
  AZ_TUNING_LIB=1 AZ_BAND_ABL=256 python tools/band_trace.py [graphs]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, ROOT)

EV = ["tile start", "A issued", "A barrier", "B edges done", "B barrier", "C MFMAs issued",
      "C partial barrier", "C barrier", "D done", "tail barrier", "tile end"]


def main():
    assert os.environ.get("AZ_TUNING_LIB") == "1" and os.environ.get("AZ_BAND_ABL") == "256"
    import torch
    import bench
    from azhip import ops, _lib
    from azhip.weights import gnn_spec, synthetic_state_dict
    graphs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = torch.device("cuda")
    Gw = synthetic_state_dict(gnn_spec(64, 2), 3)
    Wl = {k[len("layers.0."):]: torch.from_numpy(v).to(dev) for k, v in Gw.items()
          if k.startswith("layers.0.")}
    g = bench._grid_graph(ops, dev, graphs)
    x = torch.rand((g.V, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 2 - 1
    out = torch.empty_like(x)
    _, ws = ops.gnn_layer(g, x, Wl, save=False, out=out)
    L = _lib.lib()
    L.az_tuning_band_trace.restype = ctypes.c_int
    L.az_tuning_band_trace.argtypes = [ctypes.c_void_p]
    buf = np.zeros(2 * 64 * 12, np.uint64)
    runs = []
    for _ in range(5):
        ops.gnn_layer(g, x, Wl, save=False, out=out, ws=ws)
        torch.cuda.synchronize()
        assert L.az_tuning_band_trace(buf.ctypes.data) == buf.size
        runs.append(buf.reshape(2, 64, 12).astype(np.int64).copy())
    ntiles = (g.V + 63) // 64
    per = -(-ntiles // 256)
    res = {"graphs": graphs, "tiles_per_block": per, "unit": "us (median over tiles 1..per-2 and 4 launches)"}
    for w, name in ((0, "wave0"), (1, "wave4")):
        t = np.stack([r[w, 1:per - 1, :len(EV)] for r in runs[1:]])   # [launch][tile][ev]
        d = np.diff(t, axis=2) / 100.0
        tile = (t[:, :, -1] - t[:, :, 0]) / 100.0
        res[name] = {f"{EV[i]} -> {EV[i + 1]}": round(float(np.median(d[:, :, i])), 3)
                     for i in range(len(EV) - 1)}
        res[name]["tile"] = round(float(np.median(tile)), 3)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

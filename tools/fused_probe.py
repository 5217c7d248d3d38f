"""Time gnn_layer_fused_kernel alone on the config-5 shard (512 grids; GRIDS=n), 20 warm
back-to-back launches:  python tools/fused_probe.py one
    python tools/fused_probe.py sweep 0 1 2 4   # AZ_FUSED_STAGGER values, tuning build"""
import os
import sys
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))


def one():
    import numpy as np
    import torch
    import bench
    from azhip import ops
    from azhip.weights import gnn_spec, synthetic_state_dict
    dev = torch.device("cuda", 0)
    Gw = synthetic_state_dict(gnn_spec(64, 2), 3)
    Wl = {k[len("layers.0."):]: torch.from_numpy(v).to(dev) for k, v in Gw.items()
          if k.startswith("layers.0.")}
    g = bench._grid_graph(ops, dev, int(os.environ.get("GRIDS", "512")))
    x = torch.rand((g.V, 64), device=dev) * 2 - 1
    Ps = ops.gnn_source_proj(g, x, Wl)
    out = torch.empty_like(x)
    for _ in range(3):
        ops.gnn_layer_fused(g, x, Ps, Wl, out)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(20):
        ops.gnn_layer_fused(g, x, Ps, Wl, out)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) / 20 * 1e3
    print(f"stagger={os.environ.get('AZ_FUSED_STAGGER', '0')} nt={os.environ.get('AZ_FUSED_NT', '0')} "
          f"grids={os.environ.get('GRIDS', '512')} "
          f"fused_us={us:.1f}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        one()
    else:
        for m in sys.argv[2:] or ["0", "1"]:     # AZ_FUSED_STAGGER values (tuning build)
            env = dict(os.environ, AZ_FUSED_STAGGER=m, AZ_TUNING_LIB="1")
            subprocess.run([sys.executable, __file__, "one"], env=env, check=True, timeout=120)

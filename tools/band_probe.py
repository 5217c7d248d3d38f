"""Probe: the eval-mode GNN layer on the config-5 grid shard (512 32x32 grids) -- time per
az_gnn_layer_infer call (HIP events) and max |diff| vs the training path (az_gnn_layer_fwd).
  python tools/band_probe.py [graphs] [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from azhip import ops
    from azhip.weights import gnn_spec, synthetic_state_dict
    graphs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda")
    Gw = synthetic_state_dict(gnn_spec(64, 2), 3)
    Wl = {k[len("layers.0."):]: torch.from_numpy(v).to(dev) for k, v in Gw.items()
          if k.startswith("layers.0.")}
    g = bench._grid_graph(ops, dev, graphs)
    x = torch.rand((g.V, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 2 - 1
    ref, _ = ops.gnn_layer(g, x, Wl, save=True)
    out = torch.empty_like(x)
    _, ws = ops.gnn_layer(g, x, Wl, save=False, out=out)
    torch.cuda.synchronize()
    err = float((out - ref).abs().max())
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        ops.gnn_layer(g, x, Wl, save=False, out=out, ws=ws)
    e[1].record()
    torch.cuda.synchronize()
    us = e[0].elapsed_time(e[1]) / reps * 1e3
    print(f"graphs={graphs} V={g.V} band={g.band} layer_us={us:.1f} "
          f"fp32eq_tflops={73728 * g.V / us / 1e6:.1f} max_diff_vs_training={err:.3g}", flush=True)
    # the whole eval forward (PolicyValueGNN.forward_graph: layer, then layer + output_transform
    # fused) vs the training-mode forward (unfused kernels)
    from azhip.nets import PolicyValueGNN
    net = PolicyValueGNN(64, 2, device=dev, init=Gw)
    ref = net.train().forward_graph(x, g)
    net.eval()
    y = net.forward_graph(x, g)
    torch.cuda.synchronize()
    ferr = float((y - ref).abs().max())
    e[0].record()
    for _ in range(reps):
        net.forward_graph(x, g)
    e[1].record()
    torch.cuda.synchronize()
    fms = e[0].elapsed_time(e[1]) / reps
    print(f"forward_ms={fms:.3f} node_updates_per_s={2 * g.V / fms / 1e3:.4g} "
          f"max_diff_vs_training_forward={ferr:.3g}", flush=True)


if __name__ == "__main__":
    main()

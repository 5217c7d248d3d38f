"""Headline benchmark: Connect4 GNN board evaluation (BASELINE.json configs[1]).

A step = one predict_with_gnn pass (per-board semantics, Connect4GNN.py:86-120 applied to a
batch) over 512 synthetic random Connect4 boards already resident in HBM:
    fused conv trunk -> output_transform GEMM1 (+ReLU) -> GEMM2 whose split-K reduction is
    fused with the policy/value heads (az_linear_heads_fwd).
Weights are random-init (PCG64) with the reference's shapes (no checkpoint download).

    python bench.py [--gpus N --steps K --warmup W --batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N     (one rank/GPU)

Each rank evaluates its own batch (rows are independent, no collective on the data path):
value = N * B * K / max-over-ranks(time).  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))

METRIC = "board-state evals/sec (GNN fwd) + self-play games/sec, Connect4, 1/2/4/8 GPU"
F = 3136
A = 8
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 2516.6    # v_mfma_f32_32x32x16_bf16: 32 cycles/SIMD, 1024 SIMDs, 2.4 GHz
# gemm_x3 runs an fp32 product as 6 bf16 MFMA products: its fp32-equivalent ceiling
X3_PEAK_TFLOPS = round(BF16_MFMA_PEAK_TFLOPS / 6, 1)
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E spec peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 + 200 steps of the B = 512 step take ~70 ms; fewer warmup steps time the chip while its
    # clock is still ramping (profiles/r03v_warmup_probe.jsonl: warmup 10 / steps 50 -> 177 us per
    # step, warmup 200 -> 156 us, unchanged at 500 timed steps)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="untimed full steps before the warmup until this much wall time has "
                         "passed (GPU clock ramp); 0 = none")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample (rank 0, N=1 only)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-aggregate", action="store_true")
    ap.add_argument("--no-agg-extra", action="store_true",
                    help="aggregate leg: only the warm 512-grid shard (profiling passes)")
    ap.add_argument("--no-selfplay", action="store_true")
    ap.add_argument("--no-grid", action="store_true", help="skip the config-5 forward leg")
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--no-b1", action="store_true", help="skip the as-called batch-1 leg")
    ap.add_argument("--large-batch", type=int, default=65536,
                    help="extra leg at this batch (SURVEY §8d config 2); 0 = skip")
    ap.add_argument("--sp-games", type=int, default=8192,
                    help="self-play leg: games per GPU, all played in lock step (8192: 'tools/sp_sweep.py' r03o, 870 vs 762 games/s for 4096 and 848 for 12288 on one box; r02s: 4096 779 vs 2048 702)")
    ap.add_argument("--sp-sims", type=int, default=100, help="numMCTSSims (SURVEY §8d config 3)")
    ap.add_argument("--sp-threads", type=int, default=0,
                    help="host threads for the engine (0: this rank's share of the visible "
                         "cores, hostcpu.threads_per_rank)")
    ap.add_argument("--sp-check", type=int, default=4,
                    help="self-play leg: episodes of the timed run compared afterwards with the "
                         "sequential reference loop (rank 0; 'agreement')")
    ap.add_argument("--sp-lanes", type=int, default=2,
                    help="engines taking turns so host search overlaps the GPU batch")
    ap.add_argument("--sp-parallel", type=int, default=0,
                    help="games in flight at once (a finished game's slot takes the next one); "
                         "0: all sp-games at once")
    return ap.parse_args()


CALIBRATION = "profiles/r05/cpu_calibration.json"   # tools/cpu_calibration.py, build container
CPU_CHILD = "--cpu-baselines-child"


def _calibration():
    try:
        return json.load(open(os.path.join(ROOT, CALIBRATION)))
    except (OSError, ValueError):
        return {}


def cpu_baseline(W, G, seconds, B, threads, gnn=True):
    """The reference CPU path's workload on this host: the per-board forward of B-board batches
    -- GNN: extract_features -> output_transform -> heads (Connect4GNN.py:31-57 +
    gnn_utils.py:115); CNN: Connect4Net.forward (Connect4Net.py:30-60) -- as oracle/torch_ref.py's
    restatement (the same torch CPU ops as the reference, fp32, eval, no_grad) on `threads`
    torch threads, repeated for ~`seconds`.  profiles/r02_cpu_calibration.json records its time
    against the imported reference's on identical inputs and threads in the build container
    (ratio within a few %)."""
    import torch
    from oracle import torch_ref as TR
    torch.set_num_threads(threads)
    rng = np.random.default_rng(1)
    boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.float32))
    Wt = TR.params(W, torch.float32, requires_grad=False)
    Gt = TR.params({k: v for k, v in G.items() if k.startswith("output_transform")},
                   torch.float32, requires_grad=False) if gnn else None

    def run():
        with torch.no_grad():
            f = TR.c4_features(boards, Wt)
            return TR.c4_heads(TR.output_transform(f, Gt) if gnn else f, Wt)
    run()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        run()
        n += 1
    dt = time.perf_counter() - t0
    cal = _calibration().get("gnn_b512" if gnn else "cnn_b512", {})
    what = "c4_features -> output_transform -> heads" if gnn else "c4_features -> heads (CNN)"
    return {"value": n * B / dt, "unit": "board evals/s", "cores": threads, "kind": "port",
            "sample": f"{n} batches x {B} random boards, {dt:.1f} s: oracle/torch_ref.py "
                      f"(the reference's torch CPU ops: {what}), fp32, {threads} threads; "
                      f"calibration {CALIBRATION}: port / reference time = "
                      f"{cal.get('ratio_port_torch_over_reference')} on the build container"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baselines_child(spec):
    """The CPU baselines, in a fresh process (bench.py --cpu-baselines-child SPEC): started with
    the rank's full visible core set (the mask before pin_rank_to_gpu_numa narrowed it), no GPU
    context, no engine threads, torch on every visible core.  Prints one
    JSON object: gnn / cnn board baselines, the self-play loop's moves, the config-5 oracle."""
    import hostcpu
    try:
        os.sched_setaffinity(0, spec["cpus"])
    except (AttributeError, OSError):
        pass
    threads = int(spec.get("threads") or hostcpu.host_cpus())
    os.environ["OMP_NUM_THREADS"] = str(threads)
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    W = synthetic_state_dict(connect4_net_spec(7), 1)
    G = synthetic_state_dict(gnn_spec(F, 2), 2)
    sec, B = spec["seconds"], spec["B"]
    out = {"host": {"cores": threads, "affinity_cpus": len(hostcpu.affinity()),
                    "cgroup_quota": hostcpu.cgroup_cpu_quota(), "cpu_model": _cpu_model(),
                    "process": "fresh child of the bench rank, full visible mask, no GPU"}}
    out["gnn_b512"] = cpu_baseline(W, G, sec, B, threads)
    out["cnn_b512"] = cpu_baseline(W, G, min(sec, 5.0), B, threads, gnn=False)
    if spec.get("selfplay"):
        # the batch-1 loop is latency-bound: timed on every visible core AND on one torch thread
        # (the faster of the two is the baseline; profiles/r05/cpu_calibration.json
        # selfplay_by_threads: one thread is as fast or faster for the reference too)
        sps = max(sec, 20.0)              # room for one whole episode (~8-11 s on one core)
        out["selfplay"] = {str(t): selfplay_cpu_baseline(W, G, spec["sims"], sps, t)
                           for t in sorted({threads, 1}, reverse=True)}
    if spec.get("grid_seconds"):
        out["grid"] = grid_cpu_baseline(spec["grid_seconds"], threads)
    print(json.dumps(out), flush=True)


def run_cpu_baselines(cpus, seconds, B, sims, selfplay, grid_seconds):
    """Runs cpu_baselines_child in a child process (see there) and returns its results."""
    import subprocess
    spec = {"cpus": list(cpus), "seconds": seconds, "B": B, "sims": sims, "selfplay": selfplay,
            "grid_seconds": grid_seconds}
    env = dict(os.environ, OMP_NUM_THREADS=str(len(cpus)))
    import hostcpu
    if hostcpu._SET_WAIT_POLICY:      # the engine's setting, not the user's: torch's default
        env.pop("OMP_WAIT_POLICY", None)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), CPU_CHILD, json.dumps(spec)],
                       env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError("CPU baseline child failed:\n" + r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def cnn_b512_leg(torch, ev, device, B=512, reps=50):
    """SURVEY.md §8d config 2, the CNN half: Net.predict (Connect4Net.forward,
    Connect4Net.py:30-60) on a batch of B random boards resident in HBM, trunk + heads."""
    rng = np.random.default_rng(11)
    boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)).to(device)
    for _ in range(5):
        ev.evaluate(boards, gnn=False)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        ev.evaluate(boards, gnn=False)
    e[1].record()
    torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1]) / reps
    return {"batch": B, "ms_per_batch": round(ms, 4), "boards_per_s": round(B / (ms * 1e-3), 1),
            "flop_per_board": 1891008,
            "tflops": round(1891008 * B / (ms * 1e-3) / 1e12, 2),
            "note": "trunk (c4_trunk_kernel) + heads; cpu_baseline: the torch restatement "
                    "timed on this host (bench.py cpu_baselines_child)"}


def as_called_b1_leg(W, G, leaves=2000):
    """The reference's calling pattern (MCTS.py:169-174): every new leaf is a batch-1 predict
    AND a batch-1 predict_with_gnn on a host numpy int64 board, results back in host numpy --
    host<->device traffic and launch latency included (Connect4GNN.py:59-120).  Also the
    one-call form the native search uses (predict_both on one board)."""
    import torch
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    net = Connect4GNNWrapper(Connect4Game(7), selfplay_args(2))
    net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in G.items()})
    boards = np.random.default_rng(5).integers(-1, 2, size=(leaves, 7, 7)).astype(np.int64)
    for b in boards[:50]:
        net.predict(b)
        net.predict_with_gnn(b)
        net.predict_both(b[None])
    t0 = time.perf_counter()
    for b in boards:
        net.predict(b)
        net.predict_with_gnn(b)
    t_pair = (time.perf_counter() - t0) / leaves
    t0 = time.perf_counter()
    for b in boards:
        net.predict_both(b[None])
    t_both = (time.perf_counter() - t0) / leaves
    return {"leaves": leaves, "us_per_leaf_predict_and_predict_with_gnn": round(t_pair * 1e6, 2),
            "leaf_evals_per_s": round(1.0 / t_pair, 1),
            "us_per_leaf_predict_both": round(t_both * 1e6, 2),
            "note": "host numpy board in, numpy (pi, v) out per call (perf_counter around the "
                    "calls, no batching); the reference on 8 CPU threads: 153 us (predict) + "
                    "1.01 ms (predict_with_gnn) per leaf, SURVEY.md §6"}


def _grid_graph(ops, device, graphs, h=32, w=32, build=True):
    rp, cl = [0], []
    for r in range(h):
        for c in range(w):
            nb = sorted(rr * w + cc for rr, cc in ((r - 1, c), (r, c - 1), (r, c + 1), (r + 1, c))
                        if 0 <= rr < h and 0 <= cc < w)
            cl += nb
            rp.append(len(cl))
    rp, cl = np.array(rp, np.int64), np.array(cl, np.int64)
    V1, E1 = h * w, len(cl)
    g = np.arange(graphs, dtype=np.int64)
    rowptr = np.concatenate([(rp[:-1][None, :] + (g * E1)[:, None]).ravel(), [graphs * E1]])
    col = (cl[None, :] + (g * V1)[:, None]).ravel()
    if not build:
        return rowptr, col
    return ops.DeviceGraph(rowptr, col, device)


def aggregate_roofline(torch, ops, device, graphs=512, full_graphs=4096, extra=True):
    """The standalone scatter-aggregate kernel (az_gnn_aggregate_fwd) as TRAINING runs it: the
    train-mode layer (az_gnn_layer_fwd) keeps alpha / agg for the backward pass.  Eval-mode
    layers on grid graphs fuse it away (layer_roofline).  Config-5 shard per GPU (512 32x32
    grids, F = 64, dst-sorted CSR), HIP events on the launch stream:
      cold -- Infinity Cache flushed (a 512 MB read) before every timed launch (the headline);
      warm -- back-to-back launches (x, 134 MB, stays in the 256 MB Infinity Cache);
      full -- all of config 5 (4096 grids, 1.07 GB of x) on this one GPU, back-to-back."""
    def run(gr, flush=None, reps=20):
        g = _grid_graph(ops, device, gr)
        V, E, Fd = g.V, g.E, 64
        gen = torch.Generator(device=device).manual_seed(0)
        x = torch.rand((V, Fd), device=device, generator=gen) * 2 - 1
        alpha = torch.rand((E,), device=device, generator=gen)
        agg = torch.empty_like(x)
        for _ in range(3):
            ops.aggregate(g, x, alpha, agg)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        for i in range(reps):
            if flush is not None:
                flush.sum()          # a 512 MB read evicts x without leaving dirty lines
            ev[2 * i].record()
            ops.aggregate(g, x, alpha, agg)
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        ms = float(np.mean([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps)]))
        nbytes = V * Fd * 4 + E * 4 + E * 4 + (V + 1) * 4 + V * Fd * 4
        return nbytes / (ms * 1e-3) / 1e9, ms * 1e3, V, E

    flush = torch.zeros((128 << 20,), dtype=torch.float32, device=device)
    gbs, us, V, E = run(graphs, flush)
    del flush
    out = {"kernel": "aggregate_small_kernel<8,2,1,NT> (training-path layer, az_gnn_layer_fwd)",
           "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None, "avg_launch_us": round(us, 2),
           "workload": f"{graphs} 32x32 grids, V={V}, E={E}, F=64 (config-5 shard per GPU), "
                       f"Infinity Cache flushed before each launch"}
    if not extra:
        return out
    wgbs, wus, _, _ = run(graphs)
    out["warm"] = {"achieved": round(wgbs, 1), "frac": round(wgbs / HBM_PEAK_GBS, 4),
                   "avg_launch_us": round(wus, 2), "note": "back-to-back launches, x cache-warm"}
    if full_graphs:
        fgbs, fus, fV, fE = run(full_graphs, reps=10)
        out["full_config"] = {"achieved": round(fgbs, 1), "frac": round(fgbs / HBM_PEAK_GBS, 4),
                              "avg_launch_us": round(fus, 2),
                              "workload": f"{full_graphs} grids, V={fV}, E={fE} (all of config 5 "
                                          f"on one GPU)"}
    return out


BAND_PRODUCTS = 3     # gnn_layer_band_kernel's MFMA products per fp32 product (fp16 form, r04)


def layer_roofline(torch, ops, device, graphs=512, full_graphs=4096, extra=True):
    """The eval-mode GNN layer exactly as az_gnn_layer_infer runs it on the config-5 grid (what
    PolicyValueGNN.forward_graph launches): band_split_weights (147 KB of fp16 weight planes)
    + gnn_layer_band_kernel (projections, attention, normalised aggregation, gate / update MLPs,
    gated residual; x and each node's source projection once, in a rolling LDS window; nothing
    but x_out reaches HBM).  Timed per layer call with HIP events on the launch stream, Infinity
    Cache flushed before each (the headline) and back-to-back.  Algorithmic work (SURVEY.md §8d
    config 5, per layer): 73,728 FLOP per node on the matrix cores (target + source projections
    2 x 16,384, gate / update_net.0 32,768, update_net.2 8,192) + 640 FLOP per edge; bytes = x
    read (V * 256) + x_out written (V * 256) + col (4E) + rowptr (4(V+1)).  The MFMAs run fp32 in
    the fp16 form (row-scaled operands as two fp16 terms, 3 products per fp32 product on
    v_mfma_f32_32x32x16_f16, az_x3.h), so the pipe is the fp16 one (the bf16 rate)."""
    from azhip.weights import gnn_spec, synthetic_state_dict
    Gw = synthetic_state_dict(gnn_spec(64, 2), 3)
    Wl = {k[len("layers.0."):]: torch.from_numpy(v).to(device) for k, v in Gw.items()
          if k.startswith("layers.0.")}

    def run(gr, flush=None, reps=20):
        g = _grid_graph(ops, device, gr)
        V, E = g.V, g.E
        x = torch.rand((V, 64), device=device,
                       generator=torch.Generator(device=device).manual_seed(0)) * 2 - 1
        out = torch.empty_like(x)
        _, ws = ops.gnn_layer(g, x, Wl, save=False, out=out)
        ops.gnn_layer(g, x, Wl, save=False, out=out, ws=ws)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        for i in range(reps):
            if flush is not None:
                flush.sum()
            ev[2 * i].record()
            ops.gnn_layer(g, x, Wl, save=False, out=out, ws=ws)
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        us = float(np.mean([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps)])) * 1e3
        mflop = 73728 * V
        flop = mflop + 640 * E
        nbytes = V * 512 + 4 * E + 4 * (V + 1)
        del x, out
        return {"V": V, "E": E, "us": us, "flop": flop, "bytes": nbytes,
                "mfma_tflops": BAND_PRODUCTS * mflop / (us * 1e-6) / 1e12,
                "fp32_equiv_tflops": flop / (us * 1e-6) / 1e12,
                "gbs": nbytes / (us * 1e-6) / 1e9, "band": g.band}

    flush = torch.zeros((128 << 20,), dtype=torch.float32, device=device)
    c = run(graphs, flush)
    del flush
    out = {"kernel": "gnn_layer_band_kernel + band_split_weights (az_gnn_layer_infer, eval-mode "
                     "GNNLayer, band %d graph)" % c["band"],
           "bound": "mfma",
           "pipe": "fp16 (v_mfma_f32_32x32x16_f16, %d products per fp32 product)" % BAND_PRODUCTS,
           "products": BAND_PRODUCTS,
           "achieved": round(c["mfma_tflops"], 2), "peak": BF16_MFMA_PEAK_TFLOPS,
           "unit": "TFLOP/s", "frac": round(c["mfma_tflops"] / BF16_MFMA_PEAK_TFLOPS, 4),
           "fp32_equiv_tflops": round(c["fp32_equiv_tflops"], 2),
           "traffic": pmc_traffic("gnn_layer_band"), "traffic_run": pmc_run("gnn_layer_band"),
           "avg_launch_us": round(c["us"], 2), "flop_per_launch": c["flop"],
           "algorithmic_bytes": c["bytes"], "hbm_gbs_algorithmic": round(c["gbs"], 1),
           "hbm_frac_algorithmic": round(c["gbs"] / HBM_PEAK_GBS, 4),
           "workload": f"{graphs} 32x32 grids, V={c['V']}, E={c['E']}, F=64, H=128 (config-5 "
                       f"shard per GPU), Infinity Cache flushed before each launch",
           "layer_us": round(c["us"], 2)}
    if extra:
        w = run(graphs)
        out["warm"] = {"us": round(w["us"], 2), "mfma_tflops": round(w["mfma_tflops"], 2),
                       "note": "back-to-back launches, x cache-warm"}
        if full_graphs:
            f = run(full_graphs, reps=5)
            out["full_config"] = {"us": round(f["us"], 2), "mfma_tflops": round(f["mfma_tflops"], 2),
                                  "frac": round(f["mfma_tflops"] / BF16_MFMA_PEAK_TFLOPS, 4),
                                  "workload": f"{full_graphs} grids, V={f['V']} (all of config 5 "
                                              f"on one GPU)"}
    return out


def grid_forward_leg(torch, ops, device, graphs=512):
    """Config 5 end to end: PolicyValueGNN(64, 2 layers) forward over `graphs`
    32x32 grids (the per-destination generalisation of gnn_utils.py:34-117: factored attention
    GEMM, per-edge scores, CSR aggregate, gate/update GEMMs with the gated residual, then
    output_transform), random-init weights of the reference's shapes.  node-updates/s =
    V x layers / forward time (HIP events on the launch stream).  The first grid's output is
    checked against the oracle (grids are independent) before timing."""
    from azhip.nets import PolicyValueGNN
    from azhip.weights import gnn_spec, synthetic_state_dict
    from oracle import nets as O
    Gw = synthetic_state_dict(gnn_spec(64, 2), 3)
    g = _grid_graph(ops, device, graphs)
    net = PolicyValueGNN(64, 2, device=device, init=Gw).eval()
    x = torch.rand((g.V, 64), device=device,
                   generator=torch.Generator(device=device).manual_seed(0)) * 2 - 1
    y = net.forward_graph(x, g)
    one = _grid_graph(ops, "cpu", 1, build=False)
    ref = O.policy_value_gnn_csr(x[:1024].cpu().double().numpy(), one[0], one[1], Gw)
    err = float(np.abs(y[:1024].cpu().double().numpy() - ref).max())
    assert err < 1e-4, err
    for _ in range(5):                  # steady state: the previous legs flushed the caches
        net.forward_graph(x, g)         # and the clock has to come back up
    reps = 30
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        net.forward_graph(x, g)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    # 73,728 FLOP/node/layer + 640 FLOP/edge/layer + 16,384 FLOP/node output
    flop = 2 * (73728 * g.V + 640 * g.E) + 16384 * g.V
    out = {"workload": f"{graphs} 32x32 grids, V={g.V}, E={g.E}, F=64, 2 layers "
                       f"(config-5 shard per GPU)",
           "ms_per_forward": round(ms, 3), "node_updates_per_s": round(2 * g.V / (ms * 1e-3), 1),
           "unit": "node-updates/s", "gflop_per_forward": round(flop / 1e9, 2),
           "tflops": round(flop / (ms * 1e-3) / 1e12, 2), "max_abs_err_vs_oracle_grid0": err}
    return out


def grid_cpu_baseline(seconds, threads):
    """Config 5's CPU baseline: the numpy oracle's vectorised CSR restatement of
    PolicyValueGNN(64, 2 layers) over 8 32x32 grids (oracle/nets.py), fp32, for ~`seconds`."""
    from azhip.weights import gnn_spec, synthetic_state_dict
    from oracle import nets as O
    Gw = synthetic_state_dict(gnn_spec(64, 2), 3)
    n_g = 8
    rng = np.random.default_rng(0)
    xs = (rng.random((1024 * n_g, 64), dtype=np.float32) * 2 - 1)
    cg = _grid_graph(None, "cpu", n_g, build=False)
    G32 = {k: np.asarray(v, np.float32) for k, v in Gw.items()}
    O.policy_value_gnn_csr(xs, cg[0], cg[1], G32, dtype=np.float32)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.policy_value_gnn_csr(xs, cg[0], cg[1], G32, dtype=np.float32)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * 2 * 1024 * n_g / dt, 1), "unit": "node-updates/s",
            "cores": threads, "kind": "port",
            "sample": f"{n} forwards of {n_g} grids (numpy fp32 oracle, vectorised CSR "
                      f"restatement), {dt:.1f} s, BLAS on {threads} threads"}


def large_batch_leg(torch, ops, ev, device, B=65536, reps=5):
    """SURVEY §8d config 2 at B = 65,536 (B = 512 is launch-latency sized): the product path
    C4Evaluator.evaluate(gnn=True) (trunk -> az_transform_heads_fwd) per batch, and the
    output_transform.0 GEMM alone (M = B) with HIP events."""
    rng = np.random.default_rng(7)
    boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)).to(device)
    Gn = ev.gnn.params
    x = torch.empty((B, F), device=device).uniform_(0, 1)
    hid = torch.empty((B, F), device=device)
    ev.evaluate(boards, gnn=True)
    ops.linear(x, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
               act=ops.ACT_RELU, out=hid)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record()
    for _ in range(reps):
        ev.evaluate(boards, gnn=True)
    e[1].record()
    for _ in range(reps):
        ops.linear(x, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                   act=ops.ACT_RELU, out=hid)
    e[2].record()
    torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1]) / reps
    gemm_ms = e[1].elapsed_time(e[2]) / reps
    del x, hid, boards
    torch.cuda.empty_cache()
    return {"batch": B, "ms_per_batch": round(ms, 3), "boards_per_s": round(B / (ms * 1e-3), 1),
            "gemm": x3_roofline("az_gemm_f32 output_transform.0 at M = %d" % B,
                                2.0 * B * F * F, gemm_ms * 1e-3,
                                traffic=pmc_traffic("gemm_large") if B == 65536 else None,
                                traffic_run=pmc_run("gemm_large") if B == 65536 else None,
                                products=gemm_products(B))}


def gemm_products(M, N=F, K=F):
    """MFMA products per fp32 product of the product dispatch for this GEMM (az_gemm_form with
    ops.workspace's 256 MB): 3 = fp16 form, 6 = bf16 form, 1 = fp32 MFMA tile."""
    from azhip import _lib
    return int(_lib.load().az_gemm_form(M, N, K, 256 << 20))


def x3_roofline(kernel, flop, seconds, traffic=None, traffic_run=None, products=6):
    """Roofline of a split-operand GEMM call: every fp32 product runs as `products` 16-bit MFMA
    products -- 3 in the fp16 form (two fp16 terms per operand, v_mfma_f32_32x32x16_f16), 6 in the
    bf16 form (three bf16 terms, v_mfma_f32_32x32x16_bf16) -- so the pipe it is bound by is the
    dense fp16 / bf16 one (the same 2516.6 TF/s): achieved = products x 2MNK / time against that
    peak (frac <= 1 by construction).  The fp32-equivalent rate (2MNK / time, whose ceiling on
    this pipe is peak / products) is kept beside it, and so is its ratio to the fp32 MFMA peak (a
    speed-up over the native fp32 pipe, not a fraction: it exceeds 1 where the split form
    outruns v_mfma_f32_*_f32)."""
    fp32_eq = flop / seconds / 1e12
    pipe = ("fp16 (v_mfma_f32_32x32x16_f16, 3 products per fp32 product)" if products == 3 else
            "bf16 (v_mfma_f32_32x32x16_bf16, 6 products per fp32 product)")
    return {"kernel": kernel, "bound": "mfma", "pipe": pipe, "products": products,
            "achieved": round(products * fp32_eq, 2), "peak": BF16_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(products * fp32_eq / BF16_MFMA_PEAK_TFLOPS, 4),
            "traffic": traffic, "traffic_run": traffic_run,
            "avg_launch_us": round(seconds * 1e6, 2), "flop_per_launch_fp32": flop,
            "mfma_flop_per_launch": products * flop,
            "fp32_equiv_tflops": round(fp32_eq, 2),
            "split_peak_fp32_equiv": round(BF16_MFMA_PEAK_TFLOPS / products, 1),
            "speedup_vs_fp32_mfma_peak": round(fp32_eq / FP32_MFMA_PEAK_TFLOPS, 4)}


def gemm_shapes_leg(torch, ops, ev, device, Ms=(800, 1576, 3150), reps=50, warm=30):
    """output_transform.0 (one az_gemm_f32 call, Linear 3136x3136 + ReLU) at the self-play
    leg's batch sizes: 8192 lock-step games on 2 lanes put ~3,150 rows into each predict_both
    (4096 games ~1,576), the tail of a run ~800 (HIP events around each call, on the launch
    stream)."""
    Gn = ev.gnn.params
    out = []
    for M in Ms:
        x = torch.empty((M, F), device=device).uniform_(0, 1)
        y = torch.empty((M, F), device=device)
        for _ in range(warm):             # the clock settles over tens of ms (main step note)
            ops.linear(x, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                       act=ops.ACT_RELU, out=y)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        for i in range(reps):
            e[2 * i].record()
            ops.linear(x, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                       act=ops.ACT_RELU, out=y)
            e[2 * i + 1].record()
        torch.cuda.synchronize()
        us = float(np.mean([e[2 * i].elapsed_time(e[2 * i + 1]) for i in range(reps)])) * 1e3
        r = x3_roofline("az_gemm_f32 output_transform.0 at M = %d" % M, 2.0 * M * F * F,
                        us * 1e-6, products=gemm_products(M))
        row = {"M": M, "avg_call_us": r["avg_launch_us"], "frac": r["frac"],
               "fp32_equiv_tflops": r["fp32_equiv_tflops"]}
        pm = _pmc_selfplay_gemm(M)
        if pm:
            row.update(pm)
        out.append(row)
        del x, y
    return out


def _pmc_selfplay_gemm(M):
    """The committed PMC pass of the self-play GEMM at this M (profiles/pmc.json gemm_selfplay,
    tools/gpu_csk_pmc.sh): HBM bytes per dispatch of the GEMM kernel, its L2 hit rate and the
    algorithmic bytes (A + W read, C written)."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc.json")))["gemm_selfplay"]
        r = d["by_M"][str(M)]["csk"]
        # not measured by this run: a committed profile's counters, labelled with its tag
        return {"committed_pmc": {"traffic": r["hbm_bytes_per_dispatch"],
                                  "traffic_algorithmic": r["algorithmic_bytes"],
                                  "l2_hit": r.get("l2_hit"), "tag": r.get("tag", d.get("tag")),
                                  "source": "profiles/pmc.json gemm_selfplay"}}
    except (OSError, KeyError, ValueError):
        return None


def selfplay_args(sims):
    """Connect4 config 3: connect4/config.yaml + --use_gnn --numMCTSSims 100."""
    from types import SimpleNamespace
    return SimpleNamespace(numMCTSSims=sims, cpuct=1.0, tempThreshold=15, use_gnn=True,
                           expand_by=5, dropout=0.3, gnn_layers=2)


def selfplay_leg(W, G, args, device, rank):
    """Self-play games/s: `sp_games` Connect4 GNN games per GPU played in lock step (native
    MCTS engine on the host, one batched predict_both per round on the GPU)."""
    import torch
    import hostcpu
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    from selfplay import play_episodes_engine
    sa = selfplay_args(args.sp_sims)
    net = Connect4GNNWrapper(Connect4Game(7), sa)
    net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in G.items()})
    eps = list(range(rank * args.sp_games, (rank + 1) * args.sp_games))
    seeds = {e: 12345 + e for e in eps}
    lanes = getattr(args, "sp_lanes", 2)
    play_episodes_engine(Connect4Game(7), net, selfplay_args(2), eps[:8], seeds, 8,
                         threads=args.sp_threads, lanes=lanes)          # warm-up
    import nn_fallback
    nn_fallback.reset()
    st = {}
    cg0 = hostcpu.cgroup_cpu_stat()
    t0 = time.perf_counter()
    par = args.sp_parallel if getattr(args, "sp_parallel", 0) > 0 else args.sp_games
    out = play_episodes_engine(Connect4Game(7), net, sa, eps, seeds, par,
                               threads=args.sp_threads, stats=st, lanes=lanes)
    dt = time.perf_counter() - t0
    cg1 = hostcpu.cgroup_cpu_stat()
    cg = {k: cg1[k] - cg0.get(k, 0) for k in ("usage_usec", "nr_periods", "nr_throttled",
                                              "throttled_usec") if k in cg1}
    failures = nn_fallback.total()
    if failures:     # degraded play (uniform priors, v = 0) is not a throughput to report
        raise RuntimeError(f"self-play leg: {failures} network fallbacks {nn_fallback.counts()}")
    moves = sum(len(std) // 2 for std, _ in out.values())
    agreement = selfplay_agreement(net, sa, out, eps[:args.sp_check] if rank == 0 else [], seeds)
    return dt, {"games": len(out), "moves": moves, "evals": st["rows"], "rounds": st["rounds"],
                "nn_failures": failures, "agreement": agreement,
                "net_wait_s": round(st["net_s"], 3), "host_s": round(st["host_s"], 3),
                "assemble_s": round(st.get("assemble_s", 0.0), 3),
                "collect_s": round(st.get("collect_s", 0.0), 3),
                "launch_s": round(st.get("launch_s", 0.0), 3),
                "cgroup_cpu": cg or None}


class _HostOnlyNet:
    """A network that costs (almost) nothing: priors / values from a fixed function of the
    board, so the engine's host work is what gets timed (the search shape differs from the
    real network's, the per-move work does not)."""

    def predict_both(self, boards):
        n = len(boards)
        h = boards.reshape(n, -1).astype(np.float32) @ np.linspace(0.01, 0.49, 49, dtype=np.float32)
        p = np.abs(np.sin(h[:, None] + np.arange(8, dtype=np.float32))) + 0.05
        p = (p / p.sum(1, keepdims=True)).astype(np.float32)
        v = np.tanh(h * 0.3).astype(np.float32)
        return p, v, p, (0.5 * v).astype(np.float32)


def selfplay_host_only(threads, sims, games=512):
    """Host-only self-play rate (no GPU in the loop): `games` Connect4 GNN-setting episodes
    through the native engine on `threads` threads with a near-free network.  games/s per core
    is the budget figure: a node with C cores and P ranks sustains about P x min(GPU-bound
    rate, (C / P) x per-core rate)."""
    from connect4.Connect4Game import Connect4Game
    from selfplay import play_episodes_engine
    eps = list(range(games))
    st = {}
    t0 = time.perf_counter()
    out = play_episodes_engine(Connect4Game(7), _HostOnlyNet(), selfplay_args(sims), eps,
                               {e: 777 + e for e in eps}, games, threads=threads, stats=st)
    dt = time.perf_counter() - t0
    rate = len(out) / dt
    return {"games": len(out), "threads": threads, "seconds": round(dt, 2),
            "games_per_s": round(rate, 1), "games_per_s_per_core": round(rate / threads, 2),
            "assemble_s": round(st.get("assemble_s", 0.0), 3),
            "note": "native engine + example assembly only (a near-free network)"}


def selfplay_agreement(net, sa, out, sample, seeds):
    """Move agreement of a sample of the timed run's own lock-step episodes with the reference's
    sequential loop (Coach.executeEpisode after np.random.seed(seed), batch-1 predict /
    predict_with_gnn through the same HIP network), untimed: per episode, the moves whose
    (board, visit-count pi) match before the first divergence.  A lock-step row rides in a batch
    of ~1,500 and is within 1e-5 of the batch-1 row, not bit-equal, so an episode can leave the
    sequential one at a UCB near tie (tests/test_gpu_selfplay.py proves every such divergence is
    one, at this batch size)."""
    import Coach as C
    import MCTS as M
    from connect4.Connect4Game import Connect4Game
    game = Connect4Game(7)
    per = []
    for e in sample:
        coach = C.Coach.__new__(C.Coach)
        coach.game, coach.args, coach.nnet = game, sa, net
        np.random.seed(seeds[e])
        coach.mcts = M.MCTS(game, net, sa)
        std, _ = coach.executeEpisode()
        a = [(np.asarray(b).tolist(), [float(x) for x in p]) for b, p, _ in std]
        b = [(np.asarray(b).tolist(), [float(x) for x in p]) for b, p, _ in out[e][0]]
        n = min(len(a), len(b))
        k = next((i for i in range(n) if a[i] != b[i]), n)
        per.append({"episode": e, "moves": len(a) // 2, "agreeing_moves": k // 2,
                    "identical": a == b})
    moves = sum(p["moves"] for p in per)
    return {"episodes": len(per), "move_agreement": round(sum(p["agreeing_moves"] for p in per)
                                                          / max(1, moves), 4),
            "episodes_identical": sum(p["identical"] for p in per), "per_episode": per}


def train_leg(W, G, device):
    """Net.train (Connect4GNN.py:122-197) on synthetic examples: one full train() call =
    20 epochs x (CNN step on 64 sampled rows + GNN step on a 64-row star), fresh Adam per call,
    plus the Adam kernel alone over the 119.6 M GNN parameters (HBM roofline: 28 B/param =
    read p, g, m, v + write p, m, v)."""
    import torch
    from azhip import ops
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    sa = selfplay_args(2)
    sa.lr, sa.epochs, sa.batch_size = 0.001, 20, 64
    net = Connect4GNNWrapper(Connect4Game(7), sa)
    net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in G.items()})
    rng = np.random.default_rng(7)
    boards = rng.integers(-1, 2, size=(256, 7, 7)).astype(np.int64)
    pis = rng.dirichlet(np.ones(8), 256)
    zs = rng.choice([-1, 1], 256)
    ex = [(boards[i], pis[i], int(zs[i])) for i in range(256)]
    gex = [(boards[i], 1, pis[i], np.float32(0.1), pis[i], np.float32(zs[i] * 0.5), int(zs[i]))
           for i in range(128)]
    np.random.seed(0)
    net.train(ex, gex)                                  # warm-up (allocations)
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        net.train(ex, gex)
    torch.cuda.synchronize()
    train_ms = (time.perf_counter() - t0) / reps * 1e3
    P = net.gnn.params
    n = P.numel
    P.grad_flat.normal_()
    P.reset_adam()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(2):
        ops.adam(P.flat, P.grad_flat, P.m, P.v, 1e-9, 1)
    evs[0].record()
    for _ in range(10):
        ops.adam(P.flat, P.grad_flat, P.m, P.v, 1e-9, 1)
    evs[1].record()
    torch.cuda.synchronize()
    us = evs[0].elapsed_time(evs[1]) / 10 * 1e3
    gbs = 28.0 * n / (us * 1e-6) / 1e9
    return {"train_call_ms": round(train_ms, 2),
            "workload": "Connect4GNNWrapper.train: 20 epochs x (CNN step + GNN star step), "
                        "batch 64, fresh Adam, 256 std / 128 GNN synthetic examples",
            "adam_roofline": {"kernel": "adam_kernel (GNN params)", "bound": "hbm",
                              "params": n, "avg_launch_us": round(us, 1),
                              "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(gbs / HBM_PEAK_GBS, 4)}}


def train_dp_leg(W, G, device, world, rank):
    """Coach.learn's train() across P ranks (Coach.py:131-135,
    Connect4GNN.py:140-197) -- the leg that puts RCCL on a data path at N > 1: one full train()
    call (20 epochs x (CNN step + 64-row star GNN step)) per mode, each rank on its own GPU:
    * "replicas": the identical step on every rank, no collective;
    * "allreduce" + gnn_grad_sync "row0": CNN rows sharded + a 188 KB all_reduce; the GNN step's
      trunk sharded, features gathered, output_transform's 78.7 MB gradient all_reduced;
    * "allreduce" + "flat": the literal one-bucket all_reduce of the 478.6 MB GNN gradient;
    * "auto": the measured choice (wrappers._probe_train_parallel, timed on this node).
    Per mode: ms per train() call (max over ranks) and params_in_sync (bit-identical parameters
    on every rank).  Beside them, the collectives alone: one all_reduce of each payload (max over
    ranks), with the ring's bus bandwidth 2(P-1)/P x bytes / time."""
    import torch
    import torch.distributed as dist
    from azhip import dist as D
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    rng = np.random.default_rng(7)
    boards = rng.integers(-1, 2, size=(256, 7, 7)).astype(np.int64)
    pis = rng.dirichlet(np.ones(8), 256)
    zs = rng.choice([-1, 1], 256)
    ex = [(boards[i], pis[i], int(zs[i])) for i in range(256)]
    gex = [(boards[i], 1, pis[i], np.float32(0.1), pis[i], np.float32(zs[i] * 0.5), int(zs[i]))
           for i in range(128)]

    def max_ms(x):
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return round(float(t.item()), 3)

    out = {"workload": "Connect4GNNWrapper.train (20 epochs x (CNN step + GNN star step), "
                       "batch 64, fresh Adam, 256 std / 128 GNN synthetic examples) per rank",
           "world": world, "backend": dist.get_backend(), "modes": {}}
    for mode, sync in (("replicas", "row0"), ("allreduce", "row0"), ("allreduce", "flat"),
                       ("auto", "row0")):
        sa = selfplay_args(2)
        sa.lr, sa.epochs, sa.batch_size = 0.001, 20, 64
        sa.train_parallel, sa.gnn_grad_sync = mode, sync
        net = Connect4GNNWrapper(Connect4Game(7), sa)
        net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
        net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in G.items()})
        np.random.seed(0)
        net.train(ex, gex)                              # warm-up (allocations; auto: the probe)
        reps = 2
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            net.train(ex, gex)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        rec = {"train_call_ms": max_ms(ms),
               "params_in_sync": bool(D.params_in_sync(net.gnn.params.flat) and
                                      D.params_in_sync(net.nnet.params.flat))}
        if mode == "auto":
            rec["choice"] = net._tp_auto
            rec["probe"] = net.train_parallel_probe
        out["modes"][mode if mode != "allreduce" else f"allreduce_{sync}"] = rec
        if mode == "allreduce" and sync == "flat":
            P = net.gnn.params
            s, e = P.span("output_transform.")
            payloads = {"cnn_grad": net.nnet.params.grad_flat,
                        "output_transform_grad": P.grad_flat[s:e], "gnn_grad_flat": P.grad_flat}
            coll = {}
            for name, buf in payloads.items():
                D.allreduce_sum_(buf)
                ts = []
                for _ in range(3):
                    dist.barrier()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    D.allreduce_sum_(buf)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                t_ms = max_ms(float(np.median(ts)) * 1e3)
                nbytes = buf.numel() * 4
                coll[name] = {"bytes": nbytes, "all_reduce_ms": t_ms,
                              "algbw_GBs": round(nbytes / (t_ms * 1e-3) / 1e9, 2),
                              "busbw_GBs": round(2 * (world - 1) / world * nbytes /
                                                 (t_ms * 1e-3) / 1e9, 2)}
            out["all_reduce"] = coll
        del net
        torch.cuda.empty_cache()
    return out


def selfplay_cpu_baseline(W, G, sims, seconds, threads):
    """The reference's sequential loop on the host: Coach.executeEpisode over this repo's Python
    MCTS (bit-exact with the reference's, tests/test_mcts_golden.py) with oracle/torch_ref.py as
    the network behind the reference's batch-1 predict plumbing (Connect4GNN.py:59-120), torch
    on `threads` threads: moves finished in `seconds`.
    tools/cpu_calibration.py measured this loop against the imported reference's loop on the
    same whole episode (profiles/r05/cpu_calibration.json: selfplay)."""
    import torch
    import Coach as C
    import MCTS as M
    from connect4.Connect4Game import Connect4Game
    from oracle import torch_ref as TR
    torch.set_num_threads(threads)
    Wt = TR.params(W, torch.float32, requires_grad=False)
    Gt = TR.params({k: v for k, v in G.items() if k.startswith("output_transform")},
                   torch.float32, requires_grad=False)

    class PortNet:
        def _run(self, board, gnn):
            b = torch.FloatTensor(np.asarray(board).astype(np.float64)).contiguous().view(1, 7, 7)
            with torch.no_grad():
                f = TR.c4_features(b, Wt)
                lp, v = TR.c4_heads(TR.output_transform(f, Gt) if gnn else f, Wt)
            return torch.exp(lp).data.cpu().numpy()[0], v.data.cpu().numpy()[0]

        def predict(self, b):
            return self._run(b, False)

        def predict_with_gnn(self, b):
            return self._run(b, True)

    game = Connect4Game(7)
    sa = selfplay_args(sims)
    moves = 0
    t0 = time.perf_counter()
    done = 0

    class Counting(M.MCTS):
        def getActionProb_g(self, board, temp=1):
            nonlocal moves
            pi = yield from super().getActionProb_g(board, temp)
            moves += 1
            if time.perf_counter() - t0 > seconds:
                raise TimeoutError
            return pi

    coach = C.Coach.__new__(C.Coach)
    coach.game, coach.args, coach.nnet = game, sa, PortNet()
    t_done = moves_done = 0
    try:
        while True:
            np.random.seed(done)
            coach.mcts = Counting(game, coach.nnet, sa)
            coach.executeEpisode()
            done += 1
            t_done, moves_done = time.perf_counter() - t0, moves
    except TimeoutError:
        pass
    dt = time.perf_counter() - t0
    # whole episodes when at least one finished (an episode's first moves cost the most, so a
    # partial one would understate the rate); else the moves of the unfinished first episode
    return {"games_done": done, "moves": moves, "seconds": round(dt, 1),
            "whole_games_seconds": round(t_done, 2), "whole_games_moves": moves_done}


def pmc_traffic(key):
    """HBM bytes per launch from the committed PMC pass (profiles/pmc.json, written from the
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs; see profiles/README.md)."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "pmc.json")))[key][
            "hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def pmc_run(key):
    """The run tag (profiles/<tag>_*) whose PMC pass measured pmc_traffic(key)."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc.json")))
        return d[key].get("tag", d.get("tag"))
    except (OSError, KeyError, ValueError):
        return None


def _leaf_timeouts():
    from azhip import wrappers
    return wrappers.leaf_timeouts()


def main():
    args = parse()
    # before any GPU call: this rank on its GPU's NUMA node (best effort; hostcpu.py); the mask
    # before the pin is what the CPU baselines' child process gets back
    import hostcpu
    visible_cpus = hostcpu.affinity()
    pin = hostcpu.pin_rank_to_gpu_numa(int(os.environ.get("LOCAL_RANK", "0")))
    hostcpu.engine_omp_defaults()
    if not args.sp_threads:
        args.sp_threads = hostcpu.threads_per_rank()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AZ_BENCH_BACKEND=gloo rehearses the N-rank path on a box with fewer GPUs (ranks share
    # devices round-robin); the driver's multi-GPU runs use nccl = RCCL, one GPU per rank
    backend = os.environ.get("AZ_BENCH_BACKEND", "nccl")
    if world > 1:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local if world > 1 else torch.cuda.current_device())
    red_dev = device if backend == "nccl" else torch.device("cpu")
    from azhip import ops
    from azhip.nets import C4Evaluator
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict

    W = synthetic_state_dict(connect4_net_spec(7), 1)
    G = synthetic_state_dict(gnn_spec(F, 2), 2)
    ev = C4Evaluator(W, G, device=device)
    B = args.batch
    rng = np.random.default_rng(1000 + rank)
    boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)).to(device)
    Wn, Gn = ev.nnet.params, ev.gnn.params
    featbuf = torch.empty((B, F), device=device)
    h = torch.empty((B, F), device=device)
    y = torch.empty((B, F), device=device)
    logp = torch.empty((B, A), device=device)
    pi = torch.empty((B, A), device=device)
    v = torch.empty((B,), device=device)

    def step():
        # the product's batched predict_with_gnn, one az_c4_eval_fwd call: trunk (also writing
        # output_transform.0's A in the GEMM's split form) -> output_transform.0 (+ReLU; its
        # split-K reduce also splitting output_transform.2's A) -> output_transform.2, every
        # tile folding its part of y (+ bias) into the heads' dot products (y is not an output
        # of predict_with_gnn and is never stored; az_x3.h HeadsEpi) -> the heads' finalize
        ops.c4_gnn_eval(boards, Wn, Gn, feat=featbuf, hidden=h, y=y, logp=logp, pi=pi, v=v)

    def step_unfused():
        # the same network as separate calls (each GEMM splitting its own A)
        feat = ops.c4_trunk(boards, Wn, out=featbuf)
        ops.linear(feat, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                   act=ops.ACT_RELU, out=h)
        return ops.linear_heads(h, Gn["output_transform.2.weight"], Gn["output_transform.2.bias"],
                                Wn["fc_policy.weight"], Wn["fc_policy.bias"],
                                Wn["fc_value.weight"], Wn["fc_value.bias"], want_y=False)

    # correctness guard: the bench path is bit-identical to the unfused calls and to the
    # evaluator's predict_with_gnn path
    step()
    _, pi_u, v_u, _ = step_unfused()
    _, pi_ref, v_ref = ev.evaluate(boards, gnn=True)
    torch.cuda.synchronize()
    assert torch.equal(pi, pi_u) and torch.equal(v, v_u)
    assert torch.equal(pi, pi_ref) and torch.equal(v, v_ref)

    # the GPU's clock ramps over the first tens of ms of sustained work (DPM): before the W
    # warmup steps, full steps run until `--settle-ms` of wall time has passed, so that even a
    # short run (the driver's --warmup 5 --steps 20) times the steady state a loaded evaluator
    # runs at (profiles/r03v_warmup_probe.jsonl: 10 warmup steps -> 177 us per step, 200 -> 156)
    settle_steps, ts = 0, time.perf_counter()
    while (time.perf_counter() - ts) * 1e3 < args.settle_ms:
        for _ in range(20):
            step()
        settle_steps += 20
        torch.cuda.synchronize()
    settle_ms = (time.perf_counter() - ts) * 1e3
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=red_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the dominant kernel's call, output_transform.0 as a standalone az_gemm_f32 (its own A
    # split + tile kernel + split-K reduce), HIP events per call on the stream it runs on
    feat = ops.c4_trunk(boards, Wn, out=featbuf)
    for _ in range(10):
        ops.linear(feat, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                   act=ops.ACT_RELU, out=h)
    n_gemm = max(args.steps, 50)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(n_gemm)]
    for e in evs:
        e[0].record()
        ops.linear(feat, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                   act=ops.ACT_RELU, out=h)
        e[1].record()
    torch.cuda.synchronize()
    gemm_ms = [e[0].elapsed_time(e[1]) for e in evs]       # output_transform.0: one az_gemm_f32
    avg_gemm_s = float(np.mean(gemm_ms)) * 1e-3
    flop = 2.0 * B * F * F

    agg = layer = None
    if not args.no_aggregate:
        layer = layer_roofline(torch, ops, device, extra=not args.no_agg_extra)
        agg = aggregate_roofline(torch, ops, device, extra=not args.no_agg_extra)

    grid = None
    if not args.no_grid:
        grid = grid_forward_leg(torch, ops, device)
        if world > 1:
            t = torch.tensor([grid["ms_per_forward"]], device=red_dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            grid["node_updates_per_s"] = round(world * 2 * 524288 / (float(t.item()) * 1e-3), 1)
            grid["n_gpus"] = world

    cnn = cnn_b512_leg(torch, ev, device, B=B)
    if world > 1:
        t = torch.tensor([cnn["ms_per_batch"]], device=red_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cnn["boards_per_s"] = round(world * B / (float(t.item()) * 1e-3), 1)

    b1 = None
    if rank == 0 and not args.no_b1:
        b1 = as_called_b1_leg(W, G)

    large = None
    if args.large_batch > 0:
        large = large_batch_leg(torch, ops, ev, device, B=args.large_batch)

    shapes = gemm_shapes_leg(torch, ops, ev, device)
    traffic = pmc_traffic("gemm")
    if agg is not None:
        agg["traffic"] = pmc_traffic("aggregate")
        agg["traffic_run"] = pmc_run("aggregate")

    sp = None
    if not args.no_selfplay:
        if world > 1:
            dist.barrier()
        dt, sp = selfplay_leg(W, G, args, device, rank)
        if world > 1:
            t = torch.tensor([dt], device=red_dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        sp.update({"threads_per_rank": args.sp_threads,
                   "host_cores_visible": hostcpu.host_cpus(),
                   "local_world_size": hostcpu.local_world_size(), "numa_pin": pin})
        if rank == 0 and not args.no_cpu:
            sp["host_only"] = selfplay_host_only(args.sp_threads, args.sp_sims)
        sp.update({"games_per_s": round(world * sp["games"] / dt, 3),
                   "evals_per_s": round(world * sp["evals"] / dt, 1),
                   "seconds": round(dt, 2), "games_per_gpu": args.sp_games,
                   "config": "Connect4 7x7, use_gnn, numMCTSSims %d, expand_by 5, cpuct 1.0, "
                             "tempThreshold 15; native lock-step episodes (engine), %d host "
                             "threads, %d lanes"
                             % (args.sp_sims, args.sp_threads, args.sp_lanes)})

    tr = None
    if not args.no_train and rank == 0 and world == 1:
        tr = train_leg(W, G, device)
    if not args.no_train and world > 1:
        tr = train_dp_leg(W, G, device, world, rank)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # the reference CPU path's workloads on this host's visible cores, in a fresh
        # process (no GPU context, no engine threads, the mask before the NUMA pin)
        cb = run_cpu_baselines(visible_cpus, args.cpu_seconds, B, args.sp_sims,
                               sp is not None, 5.0 if grid is not None else 0.0)
        host = cb["host"]
        cpu = dict(cb["gnn_b512"], host=host)
        cnn["cpu_baseline"] = cb["cnn_b512"]
        if grid is not None:
            grid["cpu_baseline"] = cb["grid"]
        if sp is not None:
            mean_moves = sp["moves"] / max(1, sp["games"])
            by = {int(t): r for t, r in cb["selfplay"].items()}
            rates = {t: (r["games_done"] / r["whole_games_seconds"] if r["games_done"] else
                         r["moves"] / mean_moves / r["seconds"]) for t, r in by.items()}
            t_best = max(rates, key=rates.get)
            b, rate = by[t_best], rates[t_best]
            measured = (f"{b['games_done']} whole episodes ({b['whole_games_moves']} moves) in "
                        f"{b['whole_games_seconds']} s" if b["games_done"] else
                        f"{b['moves']} moves in {b['seconds']} s = {b['moves'] / mean_moves:.2f} "
                        f"games at the GPU leg's mean {mean_moves:.1f} moves/game")
            cal = _calibration()
            ratio = (cal.get("selfplay_by_threads", {}).get(str(t_best), {})
                     .get("ratio_port_over_reference_time")
                     or cal.get("selfplay", {}).get("ratio_port_over_reference_time"))
            sp["cpu_baseline"] = {
                "value": round(rate, 4), "unit": "games/s", "cores": t_best, "kind": "port",
                "reference_equivalent": round(rate * ratio, 4) if ratio else None,
                "by_threads": {str(t): round(r, 4) for t, r in sorted(rates.items())},
                "sample": f"reference sequential loop (this repo's bit-exact Python MCTS, batch-1 "
                          f"predict + predict_with_gnn through oracle/torch_ref.py with the "
                          f"reference's predict plumbing, fresh process), timed on "
                          f"{' and '.join(str(t) for t in sorted(by, reverse=True))} torch "
                          f"threads, the faster reported ({t_best}): {measured}; "
                          f"{CALIBRATION}: this loop "
                          f"takes {ratio} of the imported reference loop's time on the same "
                          f"episode at that thread count (build container) -> "
                          f"reference_equivalent",
                "host": host}

    if rank == 0:
        value = world * B * args.steps / elapsed
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "board evals/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "clock_settle": {"ms": round(settle_ms, 1), "steps": settle_steps,
                             "note": "untimed full steps before the warmup (GPU clock ramp)"},
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 (fp16x2 row-scaled split, 3 products: output_transform GEMMs and the "
                     "trunk's conv2 split each fp32 operand row, power-of-two scaled, into 2 fp16 "
                     "terms, 3 fp16 MFMA products, fp32 accumulate; ~22-bit operands: "
                     "tests/test_gpu_trained.py holds pi / v / log pi to 1e-5 of float64 and of "
                     "the reference on its trained weights, margins reported)",
            "data": "synthetic (uniform random {-1,0,1} 7x7 boards; PCG64 random-init weights "
                    "of the reference shapes)",
            "config": {"workload": "Connect4 (reference 7x7+pass board) Connect4GNN "
                                   "predict_with_gnn per-board fwd: trunk -> output_transform "
                                   "-> heads, batch of random boards per GPU",
                       "global_batch": B * world, "batch_per_gpu": B, "feature_dim": F,
                       "parallelism": f"dp{world} (independent shards, no collective)"},
            "roofline": x3_roofline(
                "az_gemm_f32 output_transform.0 as a standalone call (A's split into fp16 planes "
                "+ row scales, tile kernel on W's cached planes, split-K reduce; timed apart from "
                "the steps, which split A inside the trunk / the reduce before), Linear 3136x3136 "
                "at M = %d: fp32 operands split into 16-bit "
                "terms (%s), their cross products on the matrix cores"
                % (B, "2 fp16 terms per row-scaled operand, 3 products"
                   if gemm_products(B) == 3 else "3 bf16 terms, 6 products"),
                flop, avg_gemm_s, traffic, pmc_run("gemm"), products=gemm_products(B)),
            "gemm_shapes": shapes,
            "layer_roofline": layer,
            "cnn_b512": cnn,
            "as_called_b1": b1,
            "aggregate_roofline": agg,
            "large_batch": large,
            "grid_forward": grid,
            "selfplay": sp,
            "train": tr,
            "cpu_baseline": cpu,
            # one-launch leaf kernel hand-over timeouts (azhip/wrappers.py; each switches an
            # evaluator to the four-launch path): non-zero means degraded batch-1 / arena legs
            "leaf_timeouts": _leaf_timeouts(),
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == CPU_CHILD:
        cpu_baselines_child(json.loads(sys.argv[2]))
    else:
        main()

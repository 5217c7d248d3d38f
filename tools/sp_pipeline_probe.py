"""The self-play leg's lock-step pipeline without a profiler: per round the host times (wait,
collect, launch) and the batch's GPU span from timing events on its lane stream; prints where
the GPU idles and what the host was doing then.   python tools/sp_pipeline_probe.py [games]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    import hostcpu
    hostcpu.pin_rank_to_gpu_numa(0)
    hostcpu.engine_omp_defaults()
    import torch
    import bench
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    from selfplay import play_episodes_engine
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    games = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    sa = bench.selfplay_args(100)
    net = Connect4GNNWrapper(Connect4Game(7), sa)
    net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in
                              synthetic_state_dict(connect4_net_spec(7), 1).items()})
    net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in
                             synthetic_state_dict(gnn_spec(3136, 2), 2).items()})
    eps = list(range(games))
    seeds = {e: 12345 + e for e in eps}
    threads = hostcpu.threads_per_rank()
    play_episodes_engine(Connect4Game(7), net, bench.selfplay_args(2), eps[:8], seeds, 8,
                         threads=threads)
    st = {"timeline": []}
    t0 = time.perf_counter()
    play_episodes_engine(Connect4Game(7), net, sa, eps, seeds, games, threads=threads, stats=st)
    dt = time.perf_counter() - t0
    tl = [r for r in st["timeline"] if "gpu_start" in r]
    spans = sorted((r["gpu_start"], r["gpu_end"]) for r in tl)
    busy, end = 0.0, spans[0][0]
    for a, b in spans:
        if b > end:
            busy += b - max(a, end)
            end = b
    wall = spans[-1][1] - spans[0][0]
    gpu_time = [r["gpu_end"] - r["gpu_start"] for r in tl]
    n = np.array([r["n"] for r in tl])
    out = {"games": games, "seconds": round(dt, 3), "games_per_s": round(games / dt, 1),
           "rounds": len(tl), "wall_gpu_span_s": round(wall, 3),
           "gpu_busy_union_s": round(busy, 3), "gpu_busy_frac": round(busy / wall, 3),
           "sum_batch_span_s": round(float(np.sum(gpu_time)), 3),
           "wait_s": round(sum(r.get("wait", 0.0) for r in st["timeline"]), 3),
           "launch_s": round(sum(r.get("launch", 0.0) for r in tl), 3),
           "collect_s": st.get("collect_s"), "host_s": st.get("host_s"), "net_s": st.get("net_s")}
    # GPU span per batch by batch-size bucket (a span includes waiting behind the other lane)
    for lo, hi in ((0, 256), (256, 1024), (1024, 2048), (2048, 3072), (3072, 5000)):
        m = (n >= lo) & (n < hi)
        if m.any():
            out[f"n{lo}_{hi}"] = {"rounds": int(m.sum()),
                                  "gpu_span_ms_mean": round(float(np.mean(np.array(gpu_time)[m])) * 1e3, 3)}
    print(json.dumps(out))
    json.dump(st["timeline"], open(os.path.join(ROOT, "gpurun_out", "sp_timeline.json"), "w"))


if __name__ == "__main__":
    main()

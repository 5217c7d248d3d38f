"""CPU-baseline calibration (BASELINE.md "CPU-baseline plan" step 1): in THIS
container, time the imported reference and this repo's CPU restatements on identical inputs and
thread counts, and record the ratios.  bench.py's cpu_baseline (run on the GPU box, where the
reference does not exist) uses the restatement whose ratio is recorded here.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_calibration.py > profiles/r05/cpu_calibration.json

Legs (8 torch threads, fp32, eval mode, torch.no_grad, median of >= 10 after 3 warm-ups):
  gnn_b512  predict_with_gnn per-row semantics at B = 512 (Connect4GNN.py:31-57 +
            gnn_utils.py:115): reference extract_features -> gnn.output_transform -> heads, vs
            oracle/torch_ref.py (same torch ops) and oracle/nets.py (numpy)
  cnn_b512  Connect4Net.forward at B = 512 (Connect4Net.py:30-60), same three
  selfplay  Coach.executeEpisode (sims 100, use_gnn, expand_tree): the reference's MCTS + its
            net vs this repo's MCTS.py + the torch_ref net, the same episode (seed 0), moves/s
"""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
THREADS = 8


def med_times(*fns, reps=12, warm=3):
    """Median seconds per call of each fn, the calls interleaved round-robin so that drift in
    the container's CPU share hits every leg alike."""
    for _ in range(warm):
        for fn in fns:
            fn()
    ts = [[] for _ in fns]
    for _ in range(reps):
        for i, fn in enumerate(fns):
            t = time.perf_counter()
            fn()
            ts[i].append(time.perf_counter() - t)
    return [statistics.median(x) for x in ts]


def main():
    torch.set_num_threads(THREADS)
    sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
    sys.path.insert(0, ROOT)
    from azhip.weights import gnn_spec, synthetic_state_dict
    from oracle import nets as O
    from oracle import torch_ref as TR
    z = np.load(os.path.join(ROOT, "tests", "golden", "c4_net.npz"))
    W = {k[2:]: z[k] for k in z.files if k.startswith("w/")}
    G = synthetic_state_dict(gnn_spec(3136, 2), 1234)
    boards = np.random.default_rng(1).integers(-1, 2, size=(512, 7, 7)).astype(np.int8)

    # ---- the restatements (what bench.py runs on the GPU box)
    Wt = TR.params(W, torch.float32, requires_grad=False)
    Gt = TR.params({k: v for k, v in G.items() if k.startswith("output_transform")},
                   torch.float32, requires_grad=False)
    bt = torch.from_numpy(boards.astype(np.float32))

    def port_gnn():
        with torch.no_grad():
            return TR.c4_heads(TR.output_transform(TR.c4_features(bt, Wt), Gt), Wt)

    def port_cnn():
        with torch.no_grad():
            return TR.c4_heads(TR.c4_features(bt, Wt), Wt)

    W32 = {k: np.asarray(v, np.float32) for k, v in W.items()}
    G32 = {k: np.asarray(v, np.float32) for k, v in G.items() if k.startswith("output_transform")}

    def numpy_gnn():
        return O.c4_heads(O.policy_value_gnn_per_row(O.c4_features(boards, W32, np.float32), G32,
                                                     np.float32), W32, np.float32)

    # ---- the reference (its modules shadow this repo's same-named ones while it is timed)
    pkg = os.path.join(ROOT, "alphazero-gnn_amd")
    sys.path[:] = [p for p in sys.path if p != pkg]
    for m in [m for m in sys.modules if m.split(".")[0] in ("connect4", "Coach", "MCTS",
                                                            "gnn_utils", "Arena")]:
        sys.modules.pop(m)
    sys.path.insert(0, REF)
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game

    class A(dict):
        __getattr__ = dict.__getitem__

    args = A(lr=0.001, dropout=0.3, epochs=20, batch_size=64, use_gnn=True, gnn_layers=2,
             numMCTSSims=100, cpuct=1.0, expand_by=5, tempThreshold=15)
    game = Connect4Game(7)
    ref = Connect4GNNWrapper(game, args)
    ref.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    ref.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in G.items()})
    ref.nnet.eval()
    ref.gnn.eval()
    rb = torch.FloatTensor(boards.astype(np.float64))

    def ref_gnn():
        with torch.no_grad():
            f = ref.extract_features(rb)
            return ref.apply_policy_value_heads(ref.gnn.output_transform(f))

    def ref_cnn():
        with torch.no_grad():
            return ref.nnet(rb)

    lp_r, v_r = ref_gnn()
    lp_p, v_p = port_gnn()
    assert float((lp_r - lp_p).abs().max()) < 1e-4 and float((v_r.view(-1) - v_p).abs().max()) < 1e-4
    out = {"threads": THREADS, "container": "8-core build container (torch CPU)",
           "torch": torch.__version__}
    t_ref, t_port = med_times(ref_gnn, port_gnn)
    t_cnn_ref, t_cnn_port = med_times(ref_cnn, port_cnn)
    # numpy last and alone: OpenBLAS worker threads spin after each call and would steal the
    # cores from torch's pool if the legs were interleaved
    t_np, = med_times(numpy_gnn)
    out["gnn_b512"] = {"reference_ms": round(t_ref * 1e3, 2), "port_torch_ms": round(t_port * 1e3, 2),
                       "port_numpy_ms": round(t_np * 1e3, 2),
                       "ratio_port_torch_over_reference": round(t_port / t_ref, 3),
                       "ratio_port_numpy_over_reference": round(t_np / t_ref, 3),
                       "reference_boards_per_s": round(512 / t_ref, 1)}
    t_ref, t_port = t_cnn_ref, t_cnn_port
    out["cnn_b512"] = {"reference_ms": round(t_ref * 1e3, 2), "port_torch_ms": round(t_port * 1e3, 2),
                       "ratio_port_torch_over_reference": round(t_port / t_ref, 3),
                       "reference_boards_per_s": round(512 / t_ref, 1)}

    # ---- self-play: the same episode, reference loop vs this repo's loop, both on torch CPU
    import importlib
    ref_coach = importlib.import_module("Coach")
    ref_mcts = importlib.import_module("MCTS")
    moves_cap = 10 ** 6          # whole episodes, as bench.py's self-play baseline samples them

    def episode_rate(coach_mod, mcts_mod, net, generator=False):
        """moves/s over the whole of episode seed 0 (moves_cap is not reached; the reference's MCTS has
        getActionProb; this repo's Coach drives the generator form getActionProb_g)."""
        coach = coach_mod.Coach.__new__(coach_mod.Coach)
        coach.game, coach.args, coach.nnet = game, args, net
        count = [0]
        name = "getActionProb_g" if generator else "getActionProb"
        orig = getattr(mcts_mod.MCTS, name)

        class Stop(Exception):
            pass

        def gap(self, board, temp=1):
            if count[0] >= moves_cap:
                raise Stop
            count[0] += 1
            return orig(self, board, temp)

        def gap_g(self, board, temp=1):
            if count[0] >= moves_cap:
                raise Stop
            count[0] += 1
            return (yield from orig(self, board, temp))

        np.random.seed(0)
        coach.mcts = mcts_mod.MCTS(game, net, args)
        setattr(mcts_mod.MCTS, name, gap_g if generator else gap)
        t = time.perf_counter()
        try:
            coach.executeEpisode()
        except Stop:
            pass
        finally:
            setattr(mcts_mod.MCTS, name, orig)
        return count[0] / (time.perf_counter() - t)

    # the batch-1 loop is latency-bound: also timed on ONE torch thread (faster than 8 here)
    sp_threads = (THREADS, 1)
    ref_rates = {}
    for t in sp_threads:
        torch.set_num_threads(t)
        ref_rates[t] = max(episode_rate(ref_coach, ref_mcts, ref),
                           episode_rate(ref_coach, ref_mcts, ref))
    ref_rate = ref_rates[THREADS]
    # this repo's MCTS / Coach (MCTS.getActionProb drives the generator) with the torch_ref net
    for m in [m for m in sys.modules if m.split(".")[0] in ("connect4", "Coach", "MCTS",
                                                            "gnn_utils", "Arena")]:
        sys.modules.pop(m)
    sys.path.remove(REF)
    sys.path.insert(0, os.path.join(ROOT, "alphazero-gnn_amd"))
    my_coach = importlib.import_module("Coach")
    my_mcts = importlib.import_module("MCTS")
    assert my_mcts.__file__.startswith(ROOT)

    class PortNet:
        """The torch_ref network behind the reference's batch-1 predict plumbing
        (Connect4GNN.py:59-120: float64 -> FloatTensor, view, no_grad, exp, .cpu().numpy())."""

        def _run(self, board, gnn):
            b = torch.FloatTensor(np.asarray(board).astype(np.float64)).contiguous().view(1, 7, 7)
            with torch.no_grad():
                f = TR.c4_features(b, Wt)
                lp, v = TR.c4_heads(TR.output_transform(f, Gt) if gnn else f, Wt)
            return torch.exp(lp).data.cpu().numpy()[0], v.data.cpu().numpy()[0]

        def predict(self, board):
            return self._run(board, False)

        def predict_with_gnn(self, board):
            return self._run(board, True)

    port_rates = {}
    for t in sp_threads:
        torch.set_num_threads(t)
        port_rates[t] = max(episode_rate(my_coach, my_mcts, PortNet(), generator=True),
                            episode_rate(my_coach, my_mcts, PortNet(), generator=True))
    port_rate = port_rates[THREADS]
    torch.set_num_threads(THREADS)
    out["selfplay"] = {"config": "Connect4 7x7, use_gnn, numMCTSSims 100, expand_by 5, episode "
                                 "seed 0, the whole episode",
                       "reference_moves_per_s": round(ref_rate, 3),
                       "port_moves_per_s": round(port_rate, 3),
                       "ratio_port_over_reference_time": round(ref_rate / port_rate, 3)}
    out["selfplay_by_threads"] = {
        str(t): {"reference_moves_per_s": round(ref_rates[t], 3),
                 "port_moves_per_s": round(port_rates[t], 3),
                 "ratio_port_over_reference_time": round(ref_rates[t] / port_rates[t], 3)}
        for t in sp_threads}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

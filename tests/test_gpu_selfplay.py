"""End-to-end search parity on the MI355X (BASELINE config 3): Connect4 7x7,
use_gnn, 100 simulations, expand_tree targets -- the setting Coach.learn runs -- with the HIP
network, against the reference's own trace of the same episodes (tests/golden G6b,
mcts_c4_gnn: the reference's Connect4GNNWrapper, same weights, same per-episode seeds).

* the network on every board the reference's search visited: within 1e-5;
* the sequential reference loop (Coach.executeEpisode, batch-1 predict / predict_with_gnn) with
  the HIP network: visit counts, pi and every np.random draw per move follow the reference
  trace; a divergence is allowed only at a UCB near-tie, |u1 - u2| below what the 1e-5 network
  tolerance can move (checked at the first differing selection), and the agreement is reported;
* lock-step native engine episodes (one slot) == the sequential loop, example for example;
* lock step at production batch sizes (G = 16 / 256 / 4096 slots, the last the bench's own
  setting: ~1,500 rows per network call): a row's bits depend on the batch it rides in (selfplay.py), so 16 episodes are
  compared move by move with the sequential loop -- the engine's rows replayed through the
  reference loop reproduce its examples exactly, and every divergence must be a UCB near tie
  the 1e-5 network tolerance can flip (tests/lockstep_parity.py);
* one Coach.learn iteration (self-play on the engine, train, arena, checkpoints).

AZ_REPORT_DIR=<dir> writes the agreement reports there as JSON.
"""
import json
import math
import os
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import assert_close, GOLDEN, golden, split_weights
from test_mcts_golden import Args, _tag
from test_selfplay import _norm_gnn, _norm_std

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TOL = 1e-5
CASE = "mcts_c4_gnn"


def _report(name, obj):
    d = os.environ.get("AZ_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".json"), "w") as f:
            json.dump(obj, f, indent=1)


@pytest.fixture(scope="module")
def c4(c4_gnn_weights):
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    w = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(dropout=0.3, gnn_layers=2))
    w.nnet.load_state_dict(split_weights(golden("c4_net.npz"), "w/"))
    w.gnn.load_state_dict(c4_gnn_weights)
    return w


@pytest.fixture(scope="module")
def meta():
    return json.load(open(os.path.join(GOLDEN, CASE + ".json")))


def test_hip_outputs_on_every_visited_board(c4):
    """Every (board -> pi, v) the reference's search requested, standard and GNN, batched."""
    z = golden(CASE + ".npz")
    pi, v, _, _ = c4.predict_both(z["std_boards"].astype(np.int64))
    assert_close("G6b/predict_both/std_pi", pi, z["std_pi"], TOL)
    assert_close("G6b/predict_both/std_v", v, z["std_v"], TOL)
    _, _, gpi, gv = c4.predict_both(z["gnn_boards"].astype(np.int64))
    assert_close("G6b/predict_both/gnn_pi", gpi, z["gnn_pi"], TOL)
    assert_close("G6b/predict_both/gnn_v", gv, z["gnn_v"], TOL)


class _Recorded:
    def __init__(self, z):
        self.std = {np.asarray(b, np.int64).tobytes(): (p, v)
                    for b, p, v in zip(z["std_boards"], z["std_pi"], z["std_v"])}
        self.gnn = {np.asarray(b, np.int64).tobytes(): (p, v)
                    for b, p, v in zip(z["gnn_boards"], z["gnn_pi"], z["gnn_v"])}

    def predict(self, board):
        p, v = self.std[board.tobytes()]
        return np.array(p, np.float32), np.float32(v)

    def predict_with_gnn(self, board):
        p, v = self.gnn[board.tobytes()]
        return np.array(p, np.float32), np.float32(v)


def _sequential(game, net, args, e):
    """Coach.executeEpisode after np.random.seed(e) (the reference loop), recording per move
    the root counts / Q / pi, every np.random.choice draw, and every UCB selection with the gap
    between its best and second-best scores."""
    import Coach as C
    import MCTS as M
    coach = C.Coach.__new__(C.Coach)
    coach.game, coach.args, coach.nnet = game, args, net
    A = game.getActionSize()
    moves, choices, selects = [], [], []
    orig_choice, orig_select = np.random.choice, M.MCTS._select

    def rec_choice(*a, **k):
        r = orig_choice(*a, **k)
        choices.append(int(r))
        return r

    def rec_select(self, s):
        a = orig_select(self, s)
        us = []
        for b in range(A):
            if not self.Vs[s][b]:
                continue
            P = self.Ps[s][b]
            if (s, b) in self.Qsa:
                u = self.Qsa[(s, b)] + args.cpuct * P * math.sqrt(self.Ns[s]) / (1 + self.Nsa[(s, b)])
            else:
                u = args.cpuct * P * math.sqrt(self.Ns[s] + M.EPS)
            us.append(float(u))
        us.sort(reverse=True)
        selects.append((s, int(a), us[0] - us[1] if len(us) > 1 else math.inf, self.Ns[s]))
        return a

    np.random.choice, M.MCTS._select = rec_choice, rec_select
    try:
        np.random.seed(e)
        coach.mcts = mc = M.MCTS(game, net, args)
        orig = mc.getActionProb_g

        def gap(board, temp=1):
            pi = yield from orig(board, temp=temp)
            s = game.stringRepresentation(board)
            moves.append(dict(board=board.astype(np.int8).tolist(), temp=temp,
                              counts=[int(mc.Nsa.get((s, a), 0)) for a in range(A)],
                              q=[float(mc.Qsa[(s, a)]) if (s, a) in mc.Qsa else None
                                 for a in range(A)],
                              qtype=[_tag(mc.Qsa[(s, a)]) if (s, a) in mc.Qsa else None
                                     for a in range(A)],
                              pi=[float(x) for x in pi], choices=len(choices)))
            return pi

        mc.getActionProb_g = gap
        std, gnn = coach.executeEpisode()
    finally:
        np.random.choice, M.MCTS._select = orig_choice, orig_select
    return dict(moves=moves, choices=choices, selects=selects, std=std, gnn=gnn)


_SEQ = {}


def _hip_sequential(c4, meta, e):
    from connect4.Connect4Game import Connect4Game
    if e not in _SEQ:
        _SEQ[e] = _sequential(Connect4Game(7), c4, Args(meta["args"]), e)
    return _SEQ[e]


def test_sequential_search_with_hip_net_follows_reference(c4, meta):
    from connect4.Connect4Game import Connect4Game
    args = Args(meta["args"])
    rec = _Recorded(golden(CASE + ".npz"))
    report = []
    for ep, ref_moves in zip(meta["episodes"], meta["moves"]):
        e = ep["episode"]
        hip = _hip_sequential(c4, meta, e)
        matched, first = 0, None
        for i, ref in enumerate(ref_moves):
            if i >= len(hip["moves"]):
                first = first or {"move": i, "why": "episode ended early"}
                break
            got = hip["moves"][i]
            same = all(got[k] == ref[k] for k in ("board", "temp", "counts", "pi")) and \
                hip["choices"][:got["choices"]] == ep["choices"][:got["choices"]]
            if not same:
                first = {"move": i}
                break
            for a, b in zip(got["q"], ref["q"]):
                assert (a is None) == (b is None) and (a is None or abs(a - b) <= TOL), (e, i)
            matched += 1
        entry = {"episode": e, "reference_moves": len(ref_moves), "hip_moves": len(hip["moves"]),
                 "agreeing_moves": matched, "first_divergence": first}
        if first is None:
            assert len(hip["moves"]) == len(ref_moves)
            assert _norm_std(hip["std"]) == [tuple(x) for x in ep["std_examples"]]
            got = _norm_gnn(hip["gnn"])
            assert len(got) == len(ep["gnn_examples"])
            for a, b in zip(got, ep["gnn_examples"]):
                assert (a[0], a[1], a[2], a[4], a[6]) == (b[0], b[1], b[2], b[4], b[6])
                assert abs(a[3] - b[3]) <= TOL and abs(a[5] - b[5]) <= TOL    # values: 1e-5
        else:
            # locate the first UCB selection that differs and check it was a near-tie
            ref_run = _sequential(Connect4Game(7), rec, args, e)
            k = next(j for j, (x, y) in enumerate(zip(ref_run["selects"], hip["selects"]))
                     if x[:2] != y[:2])
            s, _, gap_ref, ns = ref_run["selects"][k]
            bound = 2.0 * (TOL + 2.0 * TOL * args.cpuct * math.sqrt(ns + 1))
            first.update(select_index=k, gap=gap_ref, bound=bound)
            assert gap_ref <= bound, entry
        report.append(entry)
    total = sum(r["reference_moves"] for r in report)
    agree = sum(r["agreeing_moves"] for r in report)
    _report("c4_gnn_sims100_sequential_agreement",
            {"case": CASE, "agreement": agree / total, "episodes": report})
    # every episode either followed the reference trace to the end or left it at a near tie
    # (asserted per episode above); the agreement itself is reported, not thresholded


def test_engine_one_slot_equals_sequential_hip(c4, meta):
    """Lock-step native engine episodes with one slot (every round a batch of one) produce the
    sequential reference loop's examples exactly, with the same HIP network."""
    from connect4.Connect4Game import Connect4Game
    from selfplay import play_episodes_engine
    eps = [ep["episode"] for ep in meta["episodes"]]
    out = play_episodes_engine(Connect4Game(7), c4, Args(meta["args"]), eps, {e: e for e in eps},
                               parallel_games=1, threads=2, lanes=1)
    for e in eps:
        hip = _hip_sequential(c4, meta, e)
        assert _norm_std(out[e][0]) == _norm_std(hip["std"]), e
        assert _norm_gnn(out[e][1]) == _norm_gnn(hip["gnn"]), e


N_COMPARED = 16      # G6c: the reference's own trace of episodes 0-15, same weights, seed = e


@pytest.mark.parametrize("G", [16, 256, 4096])
def test_lockstep_engine_parity_at_production_batches(c4, meta, G):
    """Lock-step engine self-play at G slots (2 lanes: leaf batches of ~G/2 .. G rows, the
    bench plays 4096) against the REFERENCE's own search trace of episodes 0-15 (G6c: the
    reference's MCTS.search / Coach.executeEpisode with its CPU torch network, same weights,
    seed = e; every UCB selection recorded), move by move (tests/lockstep_parity.py):
    * every compared episode's engine rows, replayed through Coach.executeEpisode, reproduce
      the engine's examples exactly (the engine's search == the reference search);
    * the rows are within 1e-5 of the batch-1 network on the same boards;
    * an episode may leave the reference's trace only at a UCB near tie the 1e-5 network
      tolerance can flip (first differing selection, the reference's own gap there <=
      near_tie_bound) -- a larger gap fails the test.  The same check against this repo's
      sequential loop with the batch-1 HIP network is kept beside it.  Agreement per episode
      with both is reported."""
    import lockstep_parity as LP
    from connect4.Connect4Game import Connect4Game
    game = Connect4Game(7)
    args = Args(meta["args"])
    trace = golden("mcts_c4_gnn_trace.npz")
    assert sorted(trace["episodes"].tolist()) == list(range(N_COMPARED))
    n = max(G, N_COMPARED)
    eps = list(range(n))
    st = {}
    out, rows = LP.record_engine_rows(game, c4, args, eps, {e: e for e in eps}, G,
                                      range(N_COMPARED), lanes=2, stats=st)
    report, worst = [], 0.0
    for e in range(N_COMPARED):
        rs = rows[e]
        boards = np.stack([r[0] for r in rs]).astype(np.int64)
        one = [c4.predict_both(boards[i:i + 1]) for i in range(len(rs))]
        for r, o in zip(rs, one):
            d = max(float(np.abs(r[1] - o[0][0]).max()), abs(float(r[2]) - float(o[1][0])),
                    float(np.abs(r[3] - o[2][0]).max()), abs(float(r[4]) - float(o[3][0])))
            worst = max(worst, d)
        ref = LP.compare_episode(game, args, e, LP.reference_trace(trace, e), rs, out[e], TOL)
        hip = LP.compare_episode(game, args, e, _hip_sequential(c4, meta, e), rs, out[e], TOL)
        ref["rows"] = len(rs)
        ref["vs_hip_sequential"] = {k: hip[k] for k in ("agreeing_moves", "divergence")}
        report.append(ref)
    moves = sum(r["moves"] for r in report)
    agree = sum(r["agreeing_moves"] for r in report)
    summary = {"G": G, "episodes_played": n, "compared": N_COMPARED,
               "against": "reference trace (G6c, mcts_c4_gnn_trace.npz)",
               "batch_rows": {"max": max(st["batch_rows"]),
                              "mean": float(np.mean(st["batch_rows"]))},
               "max_row_diff_vs_batch1": worst, "move_agreement": agree / moves,
               "episodes_identical": sum(r["divergence"] is None for r in report),
               "episodes": report}
    _report(f"c4_gnn_sims100_lockstep_parity_G{G}", summary)
    assert worst <= TOL, worst
    for r in report:
        assert r["replay_equals_engine"], r
        d = r["divergence"]
        assert d is None or d["near_tie"], r
        d = r["vs_hip_sequential"]["divergence"]
        assert d is None or d["near_tie"], r
    if G >= 256:
        assert max(st["batch_rows"]) > 64       # really ran the large-batch (x3 GEMM) path


@pytest.mark.parametrize("B", [400, 1576, 3150])
def test_predict_both_standard_heads_from_the_trunk(c4, B):
    """predict_both above 320 rows: the split-A trunk computes the standard heads from its LDS
    rows (trunk_rows_heads) -- the same bits as predict_batch, whose heads run as their own
    launch on feat (az_heads_fwd), and the GNN heads as predict_batch_with_gnn."""
    rng = np.random.default_rng(B)
    boards = rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int64)
    pi, v, gpi, gv = [np.array(x) for x in c4.predict_both_async(boards).result()]   # fused
    pi1, v1 = [np.array(x) for x in c4.predict_batch_async(boards).result()[:2]]     # separate
    assert np.array_equal(pi, pi1) and np.array_equal(v.ravel(), v1.ravel())
    # and within the 1e-5 the evaluator is held to of the torch-op path (own launches)
    pi2, v2, gpi2, gv2 = c4.predict_both(boards)
    assert_close(f"predict_both_async/std_pi/B{B}", pi, pi2, 1e-5)
    assert_close(f"predict_both_async/gnn_v/B{B}", gv.ravel(), np.asarray(gv2).ravel(), 1e-5)


def test_batch_row_bit_identity_report(c4):
    """Which batch sizes give a row the batch-1 bits (the premise of exact lock-step parity):
    rows always agree within 1e-5; bit identity is reported."""
    z = golden("c4_gnn.npz")
    boards = np.concatenate([z["boards"]] * 8).astype(np.int64)
    ref = [np.concatenate([np.asarray(x).ravel() for x in c4.predict_both(boards[i:i + 1])])
           for i in range(4)]
    rep = {}
    for B in (1, 2, 3, 4, 8, 16, 32, 64, 256, 512):
        out = c4.predict_both(boards[:B])
        rows = [np.concatenate([np.asarray(x[i]).ravel() for x in out]) for i in range(4)
                if i < B]
        for a, b in zip(rows, ref):
            np.testing.assert_allclose(a, b, atol=TOL)
        rep[B] = all(np.array_equal(a, b) for a, b in zip(rows, ref))
    _report("batch_row_bit_identity", rep)
    assert rep[1]


def test_batch_rows_up_to_8_are_batch1_bits(c4):
    """The premise of the arena's speculative leaf batches (mcts_native.ArenaPlayer,
    c4.batch_invariant_rows == 8): in any batch of <= 8 boards every row of predict_both --
    pi, v, gnn_pi, gnn_v -- is bit-identical (torch.equal) to the batch-1 evaluation of that
    board, whatever the other rows are and wherever the row sits."""
    z = golden(CASE + ".npz")
    boards = z["std_boards"].astype(np.int64)
    rng = np.random.default_rng(5)
    pick = rng.choice(len(boards), size=48, replace=False)
    one = {int(i): [torch.from_numpy(np.ascontiguousarray(np.asarray(x).reshape(-1)))
                    for x in c4.predict_both(boards[i:i + 1])] for i in pick}
    assert c4.batch_invariant_rows == 8
    for B in range(1, 9):
        for t in range(6):
            idx = rng.choice(pick, size=B, replace=False)
            out = c4.predict_both(boards[idx])
            for r, i in enumerate(idx):
                for k, x in enumerate(out):
                    row = torch.from_numpy(np.ascontiguousarray(np.asarray(x[r]).reshape(-1)))
                    assert torch.equal(row, one[int(i)][k]), (B, t, r, k)


def test_arena_speculative_batches_equal_batch1(c4):
    """Arena gating (Coach.py:137-145) with the HIP GNN players, config 3 search (sims 100):
    speculative leaf batches (leaf + children, rows cached) play exactly the games of batch-1
    leaves -- same moves, same W/L/D -- with about half the network calls."""
    from Arena import Arena
    from connect4.Connect4Game import Connect4Game
    from connect4.Connect4GNN import Connect4GNNWrapper
    from mcts_native import ArenaPlayer
    game = Connect4Game(7)
    args = SimpleNamespace(numMCTSSims=100, cpuct=1.0, use_gnn=True, dropout=0.3, gnn_layers=2)
    torch.manual_seed(11)
    other = Connect4GNNWrapper(game, args)
    res, calls = [], []
    for prefetch in (False, True):
        np.random.seed(7)
        p1 = ArenaPlayer(game, c4, args, prefetch=prefetch)
        p2 = ArenaPlayer(game, other, args, prefetch=prefetch)
        moves = []

        def rec(p):
            def f(x):
                a = p(x)
                moves.append((np.asarray(x).tobytes(), a))
                return a
            return f
        wld = Arena(rec(p1), rec(p2), game).playGames(2)
        res.append((wld, moves))
        calls.append((p1.calls + p2.calls, p1.hits + p2.hits))
    _report("arena_speculative_calls", {"batch1": calls[0], "speculative": calls[1],
                                        "wld": list(res[0][0])})
    assert res[0] == res[1]
    assert calls[1][0] < 0.7 * calls[0][0] and calls[1][0] + calls[1][1] == calls[0][0]


def test_coach_learn_connect4_gnn_sims100(tmp_path):
    """Config 3 end to end on the GPU: connect4/config.yaml + --use_gnn --numMCTSSims 100,
    self-play on the native engine (lock step), train, arena, checkpoints; no network fallback
    (checked by the autouse fixture in conftest.py)."""
    import main as M
    from Coach import Coach
    from register import get_game
    args = M.config_to_args(M.load_config(os.path.join(M.HERE, "connect4", "config.yaml")))
    args.update(numIters=1, use_gnn=True, gnn_layers=2, game="connect4", load_model=False,
                numEps=4, parallel_games=4, numMCTSSims=100, arenaCompare=2, epochs=2)
    folder = str(tmp_path / "connect4")
    os.makedirs(folder)
    args.checkpoint, args.load_folder_file = folder, (folder, "best_gnn.pth.tar")
    np.random.seed(3)
    GameClass, NNet = get_game("connect4", use_gnn=True)
    game = M.create_game_instance(GameClass, args)
    coach = Coach(game, NNet(game, args), args)
    coach.learn()
    std, gnn = coach.trainExamplesHistory[0]
    assert len(std) == 2 * len(gnn) and len(gnn) >= 4 * 7
    for b, p, r in std:
        assert b.shape == (7, 7) and abs(sum(p) - 1) < 1e-6 and abs(r) in (1, 1e-4)
    for x in gnn:
        assert len(x) == 7 and abs(np.sum(x[2]) - 1) < 1e-9 and abs(np.sum(x[4]) - 1) < 1e-9
    files = sorted(os.listdir(folder))
    assert {"best_gnn.pth.tar", "checkpoint_1_gnn.pth.tar", "checkpoint_0_gnn.pth.tar.examples",
            "temp.pth.tar"} <= set(files), files

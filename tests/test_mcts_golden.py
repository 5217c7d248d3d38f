"""Search parity (host, no GPU): this package's MCTS + Coach.executeEpisode, driven by the
network outputs the reference recorded (a lookup keyed by board bytes), must reproduce the
reference's self-play episodes bit for bit: root visit counts, root Q values and their
numeric types (np.float32 / int / float tower), returned pi, every np.random.choice draw and
the emitted training examples (tests/golden/make_goldens.py, G6).  This separates search
parity (exact) from network parity (1e-5, tests/test_gpu_*.py)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden


class RecordedNet:
    """Returns the reference's recorded (pi, v) for a board; fails on an unseen board."""

    def __init__(self, z, n):
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


def _tag(x):
    if isinstance(x, np.floating):
        return "np." + x.dtype.name
    return type(x).__name__


class Args(dict):
    def __getattr__(self, k):
        return self[k]


def run_golden(name, game, n):
    import Coach as C
    import MCTS as M
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    net = RecordedNet(golden(name + ".npz"), n)
    args = Args(meta["args"])
    coach = C.Coach.__new__(C.Coach)
    coach.game, coach.args, coach.nnet = game, args, net
    orig_choice = np.random.choice
    choices = []

    def rec_choice(*a, **k):
        r = orig_choice(*a, **k)
        choices.append(int(r))
        return r

    np.random.choice = rec_choice
    try:
        for ep_moves, ep in zip(meta["moves"], meta["episodes"]):
            np.random.seed(ep["episode"])
            coach.mcts = M.MCTS(game, net, args)
            mc = coach.mcts
            seen = []
            orig = mc.getActionProb_g

            def gap(board, temp=1, mc=mc, orig=orig, seen=seen):
                pi = yield from orig(board, temp=temp)
                s = game.stringRepresentation(board)
                A = game.getActionSize()
                seen.append(dict(
                    board=board.astype(np.int8).tolist(), temp=temp,
                    counts=[int(mc.Nsa.get((s, a), 0)) for a in range(A)],
                    q=[float(mc.Qsa[(s, a)]) if (s, a) in mc.Qsa else None for a in range(A)],
                    qtype=[_tag(mc.Qsa[(s, a)]) if (s, a) in mc.Qsa else None for a in range(A)],
                    pi=[float(x) for x in pi]))
                return pi

            mc.getActionProb_g = gap
            c0 = len(choices)
            std, gnn = coach.executeEpisode()
            assert len(seen) == len(ep_moves)
            for i, (a, b) in enumerate(zip(seen, ep_moves)):
                for key in ("board", "temp", "counts", "q", "qtype", "pi"):
                    assert a[key] == b[key], (name, ep["episode"], i, key, a[key], b[key])
            assert choices[c0:] == ep["choices"]
            assert len(mc.Ns) == ep["n_nodes"]
            assert int(sum(mc.Nsa.values())) == ep["nsa_total"]
            got_std = [(np.asarray(b).astype(int).tolist(), [float(x) for x in p], float(z))
                       for b, p, z in std]
            assert got_std == [tuple(x) for x in map(tuple, ep["std_examples"])] or \
                got_std == [(x[0], x[1], x[2]) for x in ep["std_examples"]]
            got_gnn = [(np.asarray(x[0]).astype(int).tolist(), int(x[1]),
                        [float(t) for t in x[2]], float(x[3]), [float(t) for t in x[4]],
                        float(x[5]), float(x[6])) for x in gnn]
            assert got_gnn == [tuple(x) for x in ep["gnn_examples"]]
    finally:
        np.random.choice = orig_choice


def test_connect4_selfplay_matches_reference():
    from connect4.Connect4Game import Connect4Game
    run_golden("mcts_c4", Connect4Game(7), 7)


def test_connect4_gnn_sims100_selfplay_matches_reference():
    """The north-star search setting (config 3): Connect4, use_gnn, 100 simulations,
    expand_tree targets (Coach.py:48-60, MCTS.py:60-149), three episodes."""
    from connect4.Connect4Game import Connect4Game
    run_golden("mcts_c4_gnn", Connect4Game(7), 7)


def test_tictactoe_gnn_selfplay_with_expand_tree_matches_reference():
    from tictactoe.TicTacToeGame import TicTacToeGame
    run_golden("mcts_ttt3", TicTacToeGame(3), 3)


def test_qsa_numeric_tower_present():
    """The golden traces hold a mix of np.float32 / int / float Q values;
    the comparison above checks each root Q's type, so the mix must actually be exercised."""
    meta = json.load(open(os.path.join(GOLDEN, "mcts_c4.json")))
    tags = {t for ep in meta["moves"] for m in ep for t in m["qtype"] if t}
    assert "np.float32" in tags and len(tags) >= 2, tags

"""Native MCTS engine (libaz_mcts.so) on the host, no GPU.

* rules: Connect4 / TicTacToe ended / valids / next-canonical equal the Python games on random
  reachable positions (which are differential-tested against the reference);
* np.sum emulation: NumPy's pairwise summation bit for bit;
* search parity: lock-step native self-play driven by the reference's recorded network outputs
  reproduces the reference's episodes (G6): per move the root visit counts, Q values and their
  Python types, pi, and every emitted example;
* differential fuzz: native vs the Python MCTS (golden-pinned) on pseudo-random networks, many
  seeds, both games, with and without the GNN path.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from test_mcts_golden import Args, _tag
from test_selfplay import BatchedRecordedNet, _norm_gnn, _norm_std


@pytest.fixture(scope="module", autouse=True)
def host_lib():
    from azhip.build import build_host
    build_host(verbose=False)
    import mcts_native
    return mcts_native.lib()


def _games():
    from connect4.Connect4Game import Connect4Game
    from tictactoe.TicTacToeGame import TicTacToeGame
    return [(0, 7, Connect4Game(7)), (0, 5, Connect4Game(5)), (1, 3, TicTacToeGame(3)),
            (1, 4, TicTacToeGame(4))]


def _random_positions(game, rng, count):
    out = []
    for _ in range(count):
        b, p = game.getInitBoard(), 1
        for _ in range(rng.integers(0, 60)):
            if game.getGameEnded(b, p) != 0:
                break
            v = game.getValidMoves(b, p)
            a = rng.choice(np.flatnonzero(v))
            b, p = game.getNextState(b, p, a)
        out.append(game.getCanonicalForm(b, p))
    return out


def test_rules_match_python_games(host_lib):
    import ctypes
    rng = np.random.default_rng(0)
    P = ctypes.c_void_p
    for kind, n, game in _games():
        A = game.getActionSize()
        for b in _random_positions(game, rng, 300):
            b8 = np.ascontiguousarray(b, np.int8)
            tag, val = ctypes.c_int(), ctypes.c_double()
            assert host_lib.az_game_ended(kind, n, b8.ctypes.data_as(P), ctypes.byref(tag),
                                          ctypes.byref(val)) == 0
            ref = game.getGameEnded(b, 1)
            assert (val.value, tag.value) == (float(ref), 0 if isinstance(ref, int) else 1)
            vv = np.zeros(A, np.int8)
            host_lib.az_game_valids(kind, n, b8.ctypes.data_as(P), vv.ctypes.data_as(P))
            valids = game.getValidMoves(b, 1)
            assert vv.tolist() == valids.tolist()
            for a in np.flatnonzero(valids):
                nb, pl = game.getNextState(b, 1, a)
                want = game.getCanonicalForm(nb, pl)
                out = np.zeros((n, n), np.int8)
                assert host_lib.az_game_next_canonical(kind, n, b8.ctypes.data_as(P), int(a),
                                                       out.ctypes.data_as(P)) == 0
                assert out.tolist() == want.tolist()


def test_pairwise_sum_is_numpy_sum(host_lib):
    import ctypes
    rng = np.random.default_rng(1)
    for n in (1, 2, 7, 8, 9, 10, 16, 17, 65, 129, 300):
        for _ in range(300):
            a = rng.random(n) * 10.0 ** rng.integers(-8, 8, n)
            a *= rng.random(n) < 0.8
            got = host_lib.az_np_pairwise_sum(a.ctypes.data_as(ctypes.c_void_p), n)
            assert got == float(np.sum(a))


def _native_episodes(game, net, args, eps, seeds, parallel, threads=2, per_move=None):
    from selfplay import play_episodes_native
    import mcts_native
    if per_move is not None:
        orig = mcts_native.NativeMCTS.getActionProb_g

        def gap(self, board, temp=1):
            pi = yield from orig(self, board, temp=temp)
            nsa, q, tag = self.engine.root_edges(self.slot, board)
            per_move.setdefault(self.slot, []).append(dict(
                board=board.astype(np.int8).tolist(), temp=temp, counts=nsa,
                q=[float(mcts_native.typed_q(t, x)) if t >= 0 else None for t, x in zip(tag, q)],
                qtype=[_tag(mcts_native.typed_q(t, x)) if t >= 0 else None
                       for t, x in zip(tag, q)],
                pi=[float(x) for x in pi]))
            return pi
        mcts_native.NativeMCTS.getActionProb_g = gap
    try:
        return play_episodes_native(game, net, args, eps, seeds, parallel_games=parallel,
                                    threads=threads)
    finally:
        if per_move is not None:
            mcts_native.NativeMCTS.getActionProb_g = orig


@pytest.mark.parametrize("case", ["mcts_c4", "mcts_ttt3", "mcts_c4_gnn"])
def test_native_episodes_equal_reference(case):
    from connect4.Connect4Game import Connect4Game
    from tictactoe.TicTacToeGame import TicTacToeGame
    game = TicTacToeGame(3) if case == "mcts_ttt3" else Connect4Game(7)
    meta = json.load(open(os.path.join(GOLDEN, case + ".json")))
    net = BatchedRecordedNet(golden(case + ".npz"), 0)
    eps = [ep["episode"] for ep in meta["episodes"]]
    # one slot: per-move root statistics against the reference trace, in order
    for ep, moves in zip(meta["episodes"], meta["moves"]):
        per = {}
        out = _native_episodes(game, net, Args(meta["args"]), [ep["episode"]],
                               {ep["episode"]: ep["episode"]}, 1, per_move=per)
        seen = per[0]
        assert len(seen) == len(moves)
        for i, (a, b) in enumerate(zip(seen, moves)):
            for key in ("board", "temp", "counts", "q", "qtype", "pi"):
                assert a[key] == b[key], (case, ep["episode"], i, key, a[key], b[key])
        std, gnn = out[ep["episode"]]
        assert _norm_std(std) == [tuple(x) for x in ep["std_examples"]]
        assert _norm_gnn(gnn) == [tuple(x) for x in ep["gnn_examples"]]
    # all episodes at once (lock step over slots, 3 host threads)
    out = _native_episodes(game, net, Args(meta["args"]), eps, {e: e for e in eps}, 64,
                           threads=3)
    for ep in meta["episodes"]:
        std, gnn = out[ep["episode"]]
        assert _norm_std(std) == [tuple(x) for x in ep["std_examples"]]
        assert _norm_gnn(gnn) == [tuple(x) for x in ep["gnn_examples"]]


class HashNet:
    """Deterministic pseudo-random network: (pi, v) a function of the board bytes only, with
    exact zeros and ties sprinkled in to exercise the masked / tie-break paths."""

    def __init__(self, A, salt):
        self.A, self.salt = A, salt

    def _row(self, b):
        b = np.asarray(b, np.int64)
        h = np.random.default_rng([self.salt] + [int(x) + 1 for x in b.ravel()])
        p = h.random(self.A).astype(np.float32)
        if h.random() < 0.2:
            p[h.integers(0, self.A)] = 0.0
        if h.random() < 0.1:
            p[:] = np.float32(0.25)
        p /= p.sum()
        v = np.float32(h.uniform(-1, 1))
        if h.random() < 0.05:
            v = np.float32(0.0)
        return p.astype(np.float32), v

    def predict(self, board):
        return self._row(board)

    def predict_with_gnn(self, board):
        p, v = self._row(-np.asarray(board))
        return p, np.float32(-v * 0.5)

    def predict_batch(self, boards):
        rows = [self._row(b) for b in boards]
        return np.stack([p for p, _ in rows]), np.array([v for _, v in rows], np.float32)

    def predict_both(self, boards):
        pi, v = self.predict_batch(boards)
        rows = [self.predict_with_gnn(b) for b in boards]
        return pi, v, np.stack([p for p, _ in rows]), np.array([x for _, x in rows], np.float32)


@pytest.mark.parametrize("gi", [0, 2, 3])
@pytest.mark.parametrize("use_gnn", [False, True])
def test_native_matches_python_mcts_fuzz(gi, use_gnn):
    from selfplay import play_episodes
    _, _, game = _games()[gi]
    args = Args(numMCTSSims=[7, 12, 25][gi % 3], cpuct=[1.0, 1.5, 0.7][gi % 3], tempThreshold=6,
                use_gnn=use_gnn, expand_by=3)
    net = HashNet(game.getActionSize(), 17 + gi)
    eps = list(range(6))
    seeds = {e: 1000 * gi + e for e in eps}
    py = play_episodes(game, net, args, eps, seeds, parallel_games=3)
    nat = _native_episodes(game, net, args, eps, seeds, 4, threads=2)
    for e in eps:
        assert _norm_std(nat[e][0]) == _norm_std(py[e][0]), e
        assert _norm_gnn(nat[e][1]) == _norm_gnn(py[e][1]), e


@pytest.mark.nn_failures_expected
def test_native_engine_errors_and_failed_batches():
    import nn_fallback
    from connect4.Connect4Game import Connect4Game
    from mcts_native import Engine
    from selfplay import play_episodes_engine, play_episodes_native
    eng = Engine(Connect4Game(7), 2, 1.0, False)
    b = np.zeros((7, 7), np.int8)
    eng.begin(0, b, 3)
    with pytest.raises(RuntimeError):
        eng.begin(0, b, 3)                       # still queued
    with pytest.raises(RuntimeError):
        eng.begin(5, b, 3)                       # bad slot
    k = eng.collect()
    assert k == 1 and eng.leaf_slots[0] == 0
    with pytest.raises(RuntimeError):
        eng.feed(2, np.ones((2, 8), np.float32) / 8, np.zeros(2, np.float32))
    # misshaped network outputs are rejected before any pointer reaches the C side
    with pytest.raises(ValueError):
        eng.feed(1, np.ones((1, 7), np.float32) / 7, np.zeros(1, np.float32))
    with pytest.raises(ValueError):
        eng.feed(1, np.ones((0, 8), np.float32), np.zeros(1, np.float32))
    with pytest.raises(ValueError):
        eng.feed(1, np.ones((1, 8), np.float32) / 8, None)

    class Broken:
        def predict_batch(self, boards):
            raise RuntimeError("device lost")

        def predict_both(self, boards):
            raise RuntimeError("device lost")

    args = Args(numMCTSSims=4, cpuct=1.0, tempThreshold=15, use_gnn=False)
    out = play_episodes_native(Connect4Game(7), Broken(), args, [0, 1], {0: 0, 1: 1}, 2)
    assert len(out) == 2 and all(len(std) > 0 for std, _ in out.values())
    assert nn_fallback.counts().get("selfplay.native", 0) > 0
    n0 = nn_fallback.total()
    out = play_episodes_engine(Connect4Game(7), Broken(), args, [0, 1], {0: 0, 1: 1}, 2,
                               threads=1)
    assert len(out) == 2 and nn_fallback.counts().get("selfplay.engine", 0) > 0
    assert nn_fallback.total() > n0
    # with the GNN path, expand_tree's root predict is unguarded (MCTS.py:108-113): the
    # engine aborts the episode and the driver re-raises the network's exception
    gargs = Args(numMCTSSims=4, cpuct=1.0, tempThreshold=15, use_gnn=True, expand_by=2)
    import gc
    import sys
    sw = sys.getswitchinterval()
    with pytest.raises(RuntimeError, match="device lost"):
        play_episodes_engine(Connect4Game(7), Broken(), gargs, [0], {0: 0}, 1, threads=1)
    # the lane loop's GIL switch interval and paused collector are restored on the way out
    assert gc.isenabled() and sys.getswitchinterval() == sw


def test_rng_emulation_matches_numpy_randomstate(host_lib):
    import ctypes
    rng = np.random.default_rng(3)
    for seed in (0, 1, 5, 12345, 2 ** 32 - 1):
        out = np.zeros(1500, np.int64)          # raw draws = the MT19937 key stream
        host_lib.az_rng_test(seed, 0, 1500, None, 0, out.ctypes.data)
        rs = np.random.RandomState(seed)
        assert out.tolist() == [int(x) for x in rs.randint(0, 2 ** 32, size=1500,
                                                              dtype=np.uint64)]
        d = np.zeros(700, np.float64)
        host_lib.az_rng_doubles(seed, 700, d.ctypes.data)
        assert d.tolist() == np.random.RandomState(seed).random_sample(700).tolist()
        for n in (1, 2, 3, 5, 7, 8, 10, 17):
            out = np.zeros(300, np.int64)
            host_lib.az_rng_test(seed, 1, 300, None, n, out.ctypes.data)
            rs = np.random.RandomState(seed)
            arr = np.arange(n)
            assert out.tolist() == [int(rs.choice(arr)) for _ in range(300)], (seed, n)
        for n in (8, 10, 17):
            for trial in range(5):
                p = rng.random(n) * (rng.random(n) < 0.7)
                if p.sum() == 0:
                    p[0] = 1.0
                p = [float(x) for x in p / p.sum()]
                pa = np.array(p)
                out = np.zeros(200, np.int64)
                host_lib.az_rng_test(seed, 2, 200, pa.ctypes.data, n, out.ctypes.data)
                rs = np.random.RandomState(seed)
                assert out.tolist() == [int(rs.choice(n, p=p)) for _ in range(200)], (seed, n)


@pytest.mark.parametrize("case", ["mcts_c4", "mcts_ttt3", "mcts_c4_gnn"])
def test_engine_episodes_equal_reference(case):
    """Whole episodes in the engine (episode mode) reproduce the reference's examples."""
    from connect4.Connect4Game import Connect4Game
    from tictactoe.TicTacToeGame import TicTacToeGame
    from selfplay import play_episodes_engine
    game = TicTacToeGame(3) if case == "mcts_ttt3" else Connect4Game(7)
    meta = json.load(open(os.path.join(GOLDEN, case + ".json")))
    net = BatchedRecordedNet(golden(case + ".npz"), 0)
    eps = [ep["episode"] for ep in meta["episodes"]]
    for parallel, lanes in ((1, 1), (64, 2), (3, 3)):
        out = play_episodes_engine(game, net, Args(meta["args"]), eps, {e: e for e in eps},
                                   parallel_games=parallel, threads=2, lanes=lanes)
        for ep in meta["episodes"]:
            std, gnn = out[ep["episode"]]
            assert _norm_std(std) == [tuple(x) for x in ep["std_examples"]]
            assert _norm_gnn(gnn) == [tuple(x) for x in ep["gnn_examples"]]


@pytest.mark.parametrize("gi", [0, 1, 2, 3])
@pytest.mark.parametrize("use_gnn", [False, True])
def test_engine_episodes_match_python_fuzz(gi, use_gnn):
    """Engine episodes == Python MCTS episodes (same seeds, pseudo-random networks), including
    example value types (int / float / np.float32) and pi list element types."""
    from selfplay import play_episodes, play_episodes_engine
    _, _, game = _games()[gi]
    args = Args(numMCTSSims=[7, 12, 25, 4][gi], cpuct=[1.0, 1.5, 0.7, 1.0][gi], tempThreshold=6,
                use_gnn=use_gnn, expand_by=[3, 5, 2, 1][gi])
    net = HashNet(game.getActionSize(), 31 + gi)
    eps = list(range(6))
    seeds = {e: 777 * gi + e for e in eps}
    py = play_episodes(game, net, args, eps, seeds, parallel_games=3)
    nat = play_episodes_engine(game, net, args, eps, seeds, parallel_games=4, threads=2)

    def typed(ex):
        return [tuple((type(x).__name__, np.asarray(x).tolist()) for x in row) for row in ex]
    for e in eps:
        assert typed(nat[e][0]) == typed(py[e][0]), e
        assert typed(nat[e][1]) == typed(py[e][1]), e


@pytest.mark.parametrize("use_gnn", [False, True])
def test_feed_collect_equals_feed_then_collect(use_gnn):
    """az_mcts_feed_collect (the feed inside the next collect's parallel pass) hands out the
    same leaves round by round as az_mcts_feed + az_mcts_collect, and the batched record export
    (az_mcts_episode_records) equals the per-slot az_mcts_episode_record / _targets."""
    from connect4.Connect4Game import Connect4Game
    from mcts_native import Engine
    game = Connect4Game(7)
    net = HashNet(game.getActionSize(), 5)
    S = 12
    engs = [Engine(game, S, 1.0, use_gnn) for _ in range(2)]
    for e in engs:
        for s in range(S):
            e.episode_begin(s, 900 + s, 9, 3, 6)
    ks = [e.collect(3) for e in engs]
    done = [{}, {}]
    for _ in range(5000):
        assert ks[0] == ks[1]
        assert np.array_equal(engs[0].leaf_boards[:ks[0]], engs[1].leaf_boards[:ks[1]])
        if ks[0] == 0:
            break
        out = net.predict_both(engs[0].leaf_boards[:ks[0]])
        engs[0].feed(ks[0], *out)
        for j, e in enumerate(engs):
            fin = e.episodes_finished()
            if j == 0:
                for s in fin:
                    done[0][s] = e.episode_record(s)
            else:
                for s, r in zip(fin, e.episode_records(fin)):
                    done[1][s] = r
        ks = [engs[0].collect(3), engs[1].feed_collect(ks[1], *out, threads=3)]
    for e, d in zip(engs, done):
        for s in e.episodes_finished():
            d[s] = e.episode_record(s)
    assert sorted(done[0]) == sorted(done[1]) == list(range(S))
    for s in range(S):
        a, b = done[0][s], done[1][s]
        assert sorted(a) == sorted(b)
        for key in a:
            if key == "result":
                assert type(a[key]) is type(b[key]) and a[key] == b[key]
            else:
                assert a[key].dtype == b[key].dtype and np.array_equal(a[key], b[key]), key


def test_feed_collect_small_cap_fails_before_feeding():
    """az_mcts_feed_collect with a cap below the slots that may hand out a leaf
    fails with nothing applied, so the same rows still go through a plain az_mcts_feed and the
    next collect hands out what a clean feed + collect would."""
    from connect4.Connect4Game import Connect4Game
    from mcts_native import Engine, lib
    game = Connect4Game(7)
    net = HashNet(game.getActionSize(), 5)
    S = 6
    engs = [Engine(game, S, 1.0, True) for _ in range(2)]
    for e in engs:
        for s in range(S):
            e.episode_begin(s, 300 + s, 9, 3, 6)
    k = [e.collect(2) for e in engs]
    assert k[0] == k[1] == S
    out = net.predict_both(engs[0].leaf_boards[:k[0]])
    e = engs[1]
    ptrs = e._rows_ptrs("test", k[1], *out, at_least=True)
    rc = lib().az_mcts_feed_collect(e.h, k[1], *ptrs, e._pb, e._ps, 1, 2)
    assert rc < 0
    assert "nothing was fed" in lib().az_mcts_last_error().decode()
    for x in engs:
        x.feed(S, *out)
    a, b = engs[0].collect(2), engs[1].collect(2)
    assert a == b and np.array_equal(engs[0].leaf_boards[:a], engs[1].leaf_boards[:b])

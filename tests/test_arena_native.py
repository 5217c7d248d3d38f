"""The arena (Coach.py:137-145 -> Arena.py:249-291) with native-engine players must play the
same games as the reference-shaped Python MCTS players: same moves, same W/L/D, given the same
network and np.random state.  The network here is a deterministic hash of the board (any
function of the board works: both paths see identical float32 outputs)."""
import hashlib

import numpy as np
import pytest

from test_mcts_golden import Args


class HashNet:
    def __init__(self, A, salt):
        self.A, self.salt = A, salt

    def _out(self, board, kind):
        b = np.ascontiguousarray(board, np.int8).tobytes()
        h = hashlib.blake2b(b + bytes([self.salt, kind]), digest_size=8).digest()
        r = np.random.default_rng(int.from_bytes(h, "little"))
        p = (r.random(self.A) + 0.05).astype(np.float32)
        return (p / p.sum()).astype(np.float32), np.float32(r.random() * 2 - 1)

    def predict(self, board):
        return self._out(board, 0)

    def predict_with_gnn(self, board):
        return self._out(board, 1)

    def predict_batch(self, boards):
        rows = [self.predict(b) for b in boards]
        return np.stack([p for p, _ in rows]), np.array([v for _, v in rows], np.float32)

    def predict_both(self, boards):
        pi, v = self.predict_batch(boards)
        rows = [self.predict_with_gnn(b) for b in boards]
        return pi, v, np.stack([p for p, _ in rows]), np.array([x for _, x in rows], np.float32)


def _games():
    from connect4.Connect4Game import Connect4Game
    from tictactoe.TicTacToeGame import TicTacToeGame
    return {"ttt3": (lambda: TicTacToeGame(3), 10, 8), "c4": (lambda: Connect4Game(7), 6, 4)}


class Recorder:
    def __init__(self, fn):
        self.fn, self.moves = fn, []

    def __call__(self, x):
        a = int(self.fn(x))
        self.moves.append((np.asarray(x).tobytes(), a))
        return a


@pytest.mark.parametrize("name", ["ttt3", "c4"])
@pytest.mark.parametrize("use_gnn", [False, True])
def test_native_arena_equals_python_arena(name, use_gnn):
    from Arena import Arena
    from MCTS import MCTS
    from mcts_native import ArenaPlayer
    make, sims, games = _games()[name]
    game = make()
    A = game.getActionSize()
    args = Args(numMCTSSims=sims, cpuct=1.0, use_gnn=use_gnn)
    pnet, nnet = HashNet(A, 1), HashNet(A, 2)

    results = []
    for native in (False, True):
        np.random.seed(123)
        if native:
            p1, p2 = ArenaPlayer(game, pnet, args), ArenaPlayer(game, nnet, args)
        else:
            pm, nm = MCTS(game, pnet, args), MCTS(game, nnet, args)
            p1 = lambda x: np.argmax(pm.getActionProb(x, temp=0))  # noqa: E731
            p2 = lambda x: np.argmax(nm.getActionProb(x, temp=0))  # noqa: E731
        r1, r2 = Recorder(p1), Recorder(p2)
        wld = Arena(r1, r2, game).playGames(games)
        results.append((wld, r1.moves, r2.moves))
    assert results[0][0] == results[1][0]
    assert results[0][1] == results[1][1] and results[0][2] == results[1][2]
    assert len(results[0][1]) > games          # several moves per game were really searched


class SpecHashNet(HashNet):
    """HashNet whose rows do not depend on the batch: ArenaPlayer may batch a leaf with its
    children (speculative leaf batches)."""
    batch_invariant_rows = 8

    def __init__(self, A, salt):
        super().__init__(A, salt)
        self.batches = []

    def predict_batch(self, boards):
        self.batches.append(len(boards))
        return super().predict_batch(boards)

    def predict_both(self, boards):
        self.batches.append(len(boards))
        pi, v = HashNet.predict_batch(self, boards)
        rows = [self.predict_with_gnn(b) for b in boards]
        return pi, v, np.stack([p for p, _ in rows]), np.array([x for _, x in rows], np.float32)


@pytest.mark.parametrize("name", ["ttt3", "c4"])
@pytest.mark.parametrize("use_gnn", [False, True])
def test_speculative_leaf_batches_play_the_same_games(name, use_gnn):
    """A leaf evaluated together with its children (rows cached by board) leaves every search,
    move and W/L/D of the arena unchanged, with fewer network calls."""
    from Arena import Arena
    from mcts_native import ArenaPlayer
    make, sims, games = _games()[name]
    game = make()
    A = game.getActionSize()
    args = Args(numMCTSSims=sims, cpuct=1.0, use_gnn=use_gnn)
    results, calls = [], []
    for prefetch in (False, True):
        pnet, nnet = SpecHashNet(A, 1), SpecHashNet(A, 2)
        np.random.seed(321)
        p1 = ArenaPlayer(game, pnet, args, prefetch=prefetch)
        p2 = ArenaPlayer(game, nnet, args, prefetch=prefetch)
        r1, r2 = Recorder(p1), Recorder(p2)
        wld = Arena(r1, r2, game).playGames(games)
        results.append((wld, r1.moves, r2.moves))
        calls.append((p1.calls + p2.calls, p1.hits + p2.hits,
                      max(pnet.batches + nnet.batches)))
    assert results[0] == results[1]
    (c0, h0, b0), (c1, h1, b1) = calls
    assert h0 == 0 and b0 == 1 and h1 > 0 and b1 <= 8
    assert c1 + h1 == c0 and c1 < c0


class FlakyNet(SpecHashNet):
    """Fails the first `fail` batched calls, then serves like SpecHashNet."""

    def __init__(self, A, salt, fail):
        super().__init__(A, salt)
        self.fail = fail

    def predict_both(self, boards):
        if self.fail > 0:
            self.fail -= 1
            raise RuntimeError("device lost")
        return super().predict_both(boards)

    def predict_batch(self, boards):
        if self.fail > 0:
            self.fail -= 1
            raise RuntimeError("device lost")
        return super().predict_batch(boards)


@pytest.mark.nn_failures_expected
@pytest.mark.parametrize("prefetch", [False, True])
def test_strict_failure_leaves_engine_usable(monkeypatch, prefetch):
    """Under AZ_STRICT_NN=1 a failed leaf batch raises NNFailure -- after the engine took the
    failed feed, so the same player searches on cleanly once the network recovers."""
    import nn_fallback
    from connect4.Connect4Game import Connect4Game
    from mcts_native import ArenaPlayer
    game = Connect4Game(7)
    args = Args(numMCTSSims=6, cpuct=1.0, use_gnn=True)
    net = FlakyNet(game.getActionSize(), 3, fail=1)
    p = ArenaPlayer(game, net, args, prefetch=prefetch)
    monkeypatch.setenv("AZ_STRICT_NN", "1")
    board = game.getInitBoard()
    with pytest.raises(nn_fallback.NNFailure):
        p(board)
    monkeypatch.delenv("AZ_STRICT_NN")
    b2 = game.getNextState(board, 1, 3)[0]
    a = p(game.getCanonicalForm(b2, -1))
    assert 0 <= a < game.getActionSize()

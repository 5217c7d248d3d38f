"""Game rules against the reference (G8, tests/golden/rules.npz: captured from the reference's
Connect4Game / TicTacToeGame on seeded random-play positions): the Python games of this
package and the native engine's rules (libaz_mcts.so) must agree exactly, including the
value types (int win/loss vs float 1e-4 draw) and the mirror-symmetry quirk."""
import ctypes

import numpy as np
import pytest

from conftest import golden

CASES = [("c4n7", "c4", 7), ("c4n5", "c4", 5), ("ttt3", "ttt", 3), ("ttt4", "ttt", 4)]


def _game(kind, n):
    from connect4.Connect4Game import Connect4Game
    from tictactoe.TicTacToeGame import TicTacToeGame
    return Connect4Game(n) if kind == "c4" else TicTacToeGame(n)


@pytest.mark.parametrize("name,kind,n", CASES)
def test_python_rules_match_reference(name, kind, n):
    z = golden("rules.npz")
    g = _game(kind, n)
    for i, b8 in enumerate(z[f"{name}/boards"]):
        b = b8.astype(np.int64)
        e1, e2, i1, i2 = z[f"{name}/ended"][i]
        r1, r2 = g.getGameEnded(b, 1), g.getGameEnded(b, -1)
        assert (float(r1), float(r2)) == (e1, e2), i
        assert (isinstance(r1, int), isinstance(r2, int)) == (bool(i1), bool(i2)), i
        v = g.getValidMoves(b, 1)
        assert v.dtype == np.int64 and v.tolist() == z[f"{name}/valids"][i].tolist()
        for a in np.flatnonzero(v):
            nb, pl = g.getNextState(b, 1, int(a))
            assert nb.tolist() == z[f"{name}/next"][i][a].tolist() and pl == \
                z[f"{name}/next_player"][i][a]
        pi = z[f"{name}/sym_pi"][i][0]
        sym = g.getSymmetries(b, pi)
        assert len(sym) == z[f"{name}/sym_boards"].shape[1]
        for j, (sb, sp) in enumerate(sym):
            assert np.asarray(sb).tolist() == z[f"{name}/sym_boards"][i][j].tolist()
            assert np.asarray(sp, np.float64).tolist() == z[f"{name}/sym_pi"][i][j + 1].tolist()


@pytest.mark.parametrize("name,kind,n", CASES)
def test_native_rules_match_reference(name, kind, n):
    from azhip.build import build_host
    build_host(verbose=False)
    import mcts_native
    L = mcts_native.lib()
    gk = mcts_native.GAME_CONNECT4 if kind == "c4" else mcts_native.GAME_TICTACTOE
    z = golden("rules.npz")
    P = ctypes.c_void_p
    for i, b8 in enumerate(z[f"{name}/boards"]):
        b8 = np.ascontiguousarray(b8)
        tag, val = ctypes.c_int(), ctypes.c_double()
        assert L.az_game_ended(gk, n, b8.ctypes.data, ctypes.byref(tag), ctypes.byref(val)) == 0
        e1, _, i1, _ = z[f"{name}/ended"][i]
        assert val.value == e1 and (tag.value == mcts_native.TAG_INT) == bool(i1)
        vv = np.zeros(z[f"{name}/valids"].shape[1], np.int8)
        L.az_game_valids(gk, n, b8.ctypes.data, vv.ctypes.data)
        assert vv.tolist() == z[f"{name}/valids"][i].tolist()
        for a in np.flatnonzero(vv):
            out = np.zeros((n, n), np.int8)
            assert L.az_game_next_canonical(gk, n, b8.ctypes.data, int(a), out.ctypes.data) == 0
            want = z[f"{name}/next"][i][a].astype(np.int64) * z[f"{name}/next_player"][i][a]
            assert out.tolist() == want.tolist()

"""Connect4 rules (host), behaviour-identical to the reference connect4/Connect4Game.py.

Square n x n board plus a pass action (Connect4Game.py:135-141); board[x][y] with x the column
and y the row counted from the bottom; pieces fall to the lowest empty y.  Win checks are
vectorised numpy window tests instead of Python loops (same boolean result).  Kept quirks:
  * the pass action is only legal when every column is full, and a full board is a draw
    worth 1e-4 (Connect4Game.py:154-183);
  * getSymmetries mirrors the board with np.fliplr, which on a [column][row] array flips the
    ROW (gravity) axis while pi is mirrored across columns (Connect4Game.py:208-212).
"""
import numpy as np


def _has_run(mask, w):
    """True when `mask` (bool [n, n], [column x][row y]) has w consecutive Trues along a column,
    a row or either diagonal (the four scans of Connect4Game.py:75-97), as a bitboard test:
    cell (x, y) is bit x*(n+1) + y, the extra bit per column is always 0 so no run wraps, and
    a run of w along direction step s exists iff bb & bb>>s & ... & bb>>(w-1)s != 0."""
    n = mask.shape[0]
    if w > n:
        return False
    padded = np.zeros((n, n + 1), dtype=bool)
    padded[:, :n] = mask
    bb = int.from_bytes(np.packbits(padded.ravel(), bitorder="little").tobytes(), "little")
    for s in (1, n + 1, n + 2, n):       # along y, along x, (x+1, y+1), (x+1, y-1)
        m = bb
        for k in range(1, w):
            m &= bb >> (k * s)
            if not m:
                break
        if m:
            return True
    return False


class Connect4Game:
    is_two_player = True

    def __init__(self, board_size=7):
        self.board_size = board_size

    def getInitBoard(self):
        return np.zeros((self.board_size, self.board_size), dtype=np.int64)

    def getBoardSize(self):
        return (self.board_size, self.board_size)

    def getActionSize(self):
        return self.board_size + 1

    def getNextState(self, board, player, action):
        n = self.board_size
        if action == n:                       # pass: same board object, other player
            return (board, -player)
        nb = np.copy(board)
        empty = np.flatnonzero(nb[action] == 0)
        assert empty.size > 0, "Column is full!"
        nb[action, empty[0]] = player
        return (nb, -player)

    def getValidMoves(self, board, player):
        n = self.board_size
        valids = np.zeros(n + 1, dtype=np.int64)
        open_cols = np.asarray(board)[:, n - 1] == 0
        if not open_cols.any():
            valids[-1] = 1
        else:
            valids[:n] = open_cols
        return valids

    def getGameEnded(self, board, player):
        b = np.asarray(board)
        w = min(4, self.board_size)
        if _has_run(b == player, w):
            return 1
        if _has_run(b == -player, w):
            return -1
        if (b[:, self.board_size - 1] == 0).any():
            return 0
        return 1e-4

    def getCanonicalForm(self, board, player):
        return player * board

    def getSymmetries(self, board, pi):
        n = self.board_size
        assert len(pi) == n + 1
        mirror_pi = np.copy(pi)
        mirror_pi[:n] = np.asarray(pi)[n - 1::-1] if n > 0 else mirror_pi[:n]
        return [(board, pi), (np.fliplr(board), mirror_pi)]

    def stringRepresentation(self, board):
        return board.tobytes()

    @staticmethod
    def display(board):
        n = board.shape[1]
        cols = " ".join(str(j) for j in range(n))
        print("  " + cols + " ")
        print(" +" + "--" * n + "+")
        for i in range(n - 1, -1, -1):
            row = "".join({-1: "O ", 1: "X "}.get(int(board[j][i]), ". ") for j in range(n))
            print(f"{i}|{row}|")
        print(" +" + "--" * n + "+")
        print("  " + cols + " ")

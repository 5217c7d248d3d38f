"""TicTacToe rules (host), behaviour-identical to the reference tictactoe/TicTacToeGame.py:
n x n board, n in a row wins (rows, columns and the two main diagonals only,
TicTacToeGame.py:60-107), pass action n*n only when the board is full, draw 1e-4, the 8
dihedral symmetries in the reference's order (rot90 by 1..4, each flipped then not)."""
import numpy as np


class TicTacToeGame:
    is_two_player = True

    def __init__(self, n=3):
        self.n = n

    def getInitBoard(self):
        return np.zeros((self.n, self.n), dtype=np.int64)

    def getBoardSize(self):
        return (self.n, self.n)

    def getActionSize(self):
        return self.n * self.n + 1

    def getNextState(self, board, player, action):
        n = self.n
        if action == n * n:
            return (board, -player)
        nb = np.copy(board)
        x, y = int(action / n), action % n
        assert nb[x][y] == 0
        nb[x][y] = player
        return (nb, -player)

    def getValidMoves(self, board, player):
        n = self.n
        valids = np.zeros(n * n + 1, dtype=np.int64)
        empty = (np.asarray(board) == 0).reshape(-1)        # index n*x + y
        if not empty.any():
            valids[-1] = 1
        else:
            valids[:-1] = empty
        return valids

    def _wins(self, b, color):
        m = b == color
        return bool(m.all(axis=0).any() or m.all(axis=1).any() or np.diagonal(m).all()
                    or np.diagonal(m[:, ::-1]).all())

    def getGameEnded(self, board, player):
        b = np.asarray(board)
        if self._wins(b, player):
            return 1
        if self._wins(b, -player):
            return -1
        if (b == 0).any():
            return 0
        return 1e-4

    def getCanonicalForm(self, board, player):
        return player * board

    def getSymmetries(self, board, pi):
        n = self.n
        assert len(pi) == n * n + 1
        pi_board = np.reshape(pi[:-1], (n, n))
        out = []
        for k in range(1, 5):
            rb, rp = np.rot90(board, k), np.rot90(pi_board, k)
            for flip in (True, False):
                b2, p2 = (np.fliplr(rb), np.fliplr(rp)) if flip else (rb, rp)
                out.append((b2, list(p2.ravel()) + [pi[-1]]))
        return out

    def stringRepresentation(self, board):
        return board.tobytes()

    @staticmethod
    def display(board):
        n = board.shape[0]
        print("   " + " ".join(str(y) for y in range(n)) + " ")
        print("  " + "--" * n + "--")
        for y in range(n):
            cells = "".join({-1: "O ", 1: "X "}.get(int(board[y][x]), "- ") for x in range(n))
            print(f"{y} |{cells}|")
        print("  " + "--" * n + "--")

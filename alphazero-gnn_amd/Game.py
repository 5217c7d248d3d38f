"""Game plugin interface (reference Game.py:1-112).

Documentation-only base class, as in the reference: implementations are duck-typed and need
not inherit it.  Boards are numpy arrays; `player` is 1 or -1; actions are ints in
[0, getActionSize()).  Connect4Game and TicTacToeGame in this package implement it."""


class Game:
    def getInitBoard(self):
        """Starting board (numpy array)."""
        raise NotImplementedError

    def getBoardSize(self):
        """(x, y) board dimensions."""
        raise NotImplementedError

    def getActionSize(self):
        """Number of actions (including a pass move where the game has one)."""
        raise NotImplementedError

    def getNextState(self, board, player, action):
        """(nextBoard, nextPlayer) after `player` plays `action`; `board` is not mutated."""
        raise NotImplementedError

    def getValidMoves(self, board, player):
        """Binary vector of length getActionSize()."""
        raise NotImplementedError

    def getGameEnded(self, board, player):
        """0 while running, 1 if `player` won, -1 if lost, a small non-zero value on a draw."""
        raise NotImplementedError

    def getCanonicalForm(self, board, player):
        """Board from `player`'s point of view (player * board for two-player games)."""
        raise NotImplementedError

    def getSymmetries(self, board, pi):
        """List of (board, pi) pairs equivalent under the game's symmetries."""
        raise NotImplementedError

    def stringRepresentation(self, board):
        """Hashable key of a board (the MCTS dictionaries are keyed by it)."""
        raise NotImplementedError

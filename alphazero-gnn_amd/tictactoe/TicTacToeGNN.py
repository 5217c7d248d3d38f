"""Drop-in for tictactoe/TicTacToeGNN.py."""
from azhip.nets import TicTacToeNet
from azhip.wrappers import GNNWrapperMixin, NetWrapper


class TicTacToeGNNWrapper(GNNWrapperMixin, NetWrapper):
    """tictactoe/TicTacToeGNN.py:9-181."""

    net_class = TicTacToeNet

"""Drop-in for tictactoe/TicTacToeNet.py."""
from azhip.nets import TicTacToeNet  # noqa: F401
from azhip.wrappers import CNNWrapperMixin, NetWrapper


class TicTacToeNNetWrapper(CNNWrapperMixin, NetWrapper):
    """tictactoe/TicTacToeNet.py:50-104."""

    net_class = TicTacToeNet

"""Drop-in for connect4/Connect4Net.py: the Connect4 CNN and its NeuralNet wrapper."""
from azhip.nets import Connect4Net  # noqa: F401
from azhip.wrappers import CNNWrapperMixin, NetWrapper


class Connect4NNetWrapper(CNNWrapperMixin, NetWrapper):
    """connect4/Connect4Net.py:62-147 (save does not create the folder, :136-141)."""

    net_class = Connect4Net
    makedirs_on_save = False

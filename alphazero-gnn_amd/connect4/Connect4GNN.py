"""Drop-in for connect4/Connect4GNN.py: Connect4 CNN + PolicyValueGNN wrapper."""
from azhip.nets import Connect4Net
from azhip.wrappers import GNNWrapperMixin, NetWrapper


class Connect4GNNWrapper(GNNWrapperMixin, NetWrapper):
    """connect4/Connect4GNN.py:14-220."""

    net_class = Connect4Net

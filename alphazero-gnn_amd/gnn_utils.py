"""Drop-in for the reference gnn_utils.py: GNNLayer / PolicyValueGNN with the same constructor
signatures and state_dict keys, computing on the MI355X through libaz_hip (azhip.nets)."""
from azhip.nets import GNNLayer, PolicyValueGNN  # noqa: F401


class GNNProcessor(PolicyValueGNN):
    """gnn_utils.py:76-85 (unused by the reference): the layer stack without output_transform."""

    def __call__(self, features):
        x = features
        if x.shape[0] > 1:
            x = self.run_layers(x, self._star(x.shape[0]))
        return x

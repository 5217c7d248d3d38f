"""NeuralNet plugin interface (reference Net.py:1-61).

Documentation-only base class, as in the reference.  The wrappers in connect4/ and tictactoe/
implement it on libaz_hip (azhip/wrappers.py) and add the batched entry points
predict_batch / predict_batch_with_gnn / predict_both used by lock-step self-play."""


class NeuralNet:
    def __init__(self, game, args):
        pass

    def train(self, examples, gnn_examples=None):
        """examples: [(board, pi, v)]; gnn_examples: [(board, player, init_pi, init_v,
        expanded_pi, expanded_v, reward)].  Updates the parameters in place."""
        raise NotImplementedError

    def predict(self, board):
        """(pi float32[A], v float32) for one canonical board."""
        raise NotImplementedError

    def predict_with_gnn(self, board):
        """Same contract, through the GNN's output transform (GNN wrappers only)."""
        raise NotImplementedError

    def save_checkpoint(self, folder, filename):
        raise NotImplementedError

    def load_checkpoint(self, folder, filename):
        raise NotImplementedError

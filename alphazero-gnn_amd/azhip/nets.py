"""The reference's networks on libaz_hip: same constructor signatures, attribute names and
state_dict keys as connect4/Connect4Net.py, tictactoe/TicTacToeNet.py and gnn_utils.py, with
parameters in one flat HBM buffer per network and every forward running as HIP kernels."""
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib, ops
from .params import FlatParams
from .weights import connect4_net_spec, gnn_spec, tictactoe_net_spec, torch_default_init


def default_device():
    _lib.lib()  # raises when no gfx950 device / library: there is no CPU fallback
    return torch.device("cuda", torch.cuda.current_device())


def _args_get(args, name, default):
    try:
        return args[name] if isinstance(args, dict) else getattr(args, name)
    except (KeyError, AttributeError):
        return default


def boards_to_device(boards, device):
    """Caller-owned boards (np int64/int8 [B,n,n] or [n,n], values in {-1,0,1}) -> int8 on HBM.
    The reference converts int64 -> float64 -> float32 (Connect4GNN.py:70); int8 carries the
    same exact values in 1/8 of the bytes."""
    if isinstance(boards, torch.Tensor):
        t = boards.to(device=device, dtype=torch.int8)
    else:
        a = np.asarray(boards)
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int8)).to(device)
    return t


class _Net:
    """nn.Module-like surface the reference's wrappers use: state_dict / load_state_dict /
    train / eval / parameters / training."""

    def state_dict(self):
        return self.params.state_dict()

    def load_state_dict(self, sd, strict=True):
        self.params.load_state_dict(sd, strict)

    def train(self, mode=True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    def parameters(self):
        return iter(self.params.views.values())

    def to(self, device):
        if torch.device(device) != self.params.device:
            raise ValueError("parameters live in one flat HBM buffer; construct on the target device")
        return self


class Connect4Net(_Net):
    """connect4/Connect4Net.py:7-60: conv1 3x3 p1 -> ReLU -> conv2 3x3 p1 -> ReLU -> flatten ->
    dropout (train only) -> fc_policy -> log_softmax ; fc_value -> tanh."""

    def __init__(self, game, args, device=None, init=None):
        self.board_x, self.board_y = game.getBoardSize()
        self.action_size = game.getActionSize()
        self.args = args
        self.dropout = _args_get(args, "dropout", 0.3)
        self.n = self.board_x
        self.feature_dim = 64 * self.board_x * self.board_y
        spec = connect4_net_spec(self.n, self.action_size)
        self.params = FlatParams(spec, device or default_device(),
                                 init if init is not None else torch_default_init(spec))
        self.training = True

    def features(self, b):
        """b: int8 [B,n,n] on HBM -> [B, 64*n*n] (Connect4Net.py:42-49)."""
        W = self.params
        W.sync()
        if self.n == 7:
            return ops.c4_trunk(b, W)
        s = ops.conv3x3_relu(b, W["conv1.weight"], W["conv1.bias"], 1)
        s = ops.conv3x3_relu(s, W["conv2.weight"], W["conv2.bias"], 1)
        return s.view(s.shape[0], -1)

    def features_heads(self, b, pi=None, v=None):
        """features(b) and heads of them -> (feat, logp, pi, v); one launch for small B on the
        7x7 board (ops.c4_trunk_heads), bit-identical to the two calls."""
        if self.n != 7:
            f = self.features(b)
            return (f,) + self.heads(f, pi=pi, v=v)
        self.params.sync()
        return ops.c4_trunk_heads(b, self.params, pi=pi, v=v)

    def heads(self, feat, want_pi=True, pi=None, v=None):
        """Connect4GNN.py:48-57 (pi / v: optional output buffers, e.g. HostBuffer views)."""
        W = self.params
        W.sync()
        return ops.heads(feat, W["fc_policy.weight"], W["fc_policy.bias"], W["fc_value.weight"],
                         W["fc_value.bias"], want_pi=want_pi, pi=pi, v=v)

    def __call__(self, b):
        logp, _, v = self.heads(self.features(b), want_pi=False)
        return logp, v.view(-1, 1)


class TicTacToeNet(_Net):
    """tictactoe/TicTacToeNet.py:8-48 (conv3 without padding, 512-wide heads, no dropout)."""

    def __init__(self, game, args, device=None, init=None):
        self.board_x, self.board_y = game.getBoardSize()
        self.action_size = game.getActionSize()
        self.args = args
        self.n = self.board_x
        self.feature_dim = 128 * (self.board_x - 2) * (self.board_y - 2)
        spec = tictactoe_net_spec(self.n, self.action_size)
        self.params = FlatParams(spec, device or default_device(),
                                 init if init is not None else torch_default_init(spec))
        self.training = True

    def features(self, b):
        W = self.params
        W.sync()
        s = ops.conv3x3_relu(b, W["conv1.weight"], W["conv1.bias"], 1)
        s = ops.conv3x3_relu(s, W["conv2.weight"], W["conv2.bias"], 1)
        s = ops.conv3x3_relu(s, W["conv3.weight"], W["conv3.bias"], 0)
        return s.view(s.shape[0], -1)

    def hidden(self, feat):
        W = self.params
        W.sync()
        h1 = ops.linear(feat, W["fc1.weight"], W["fc1.bias"], act=ops.ACT_RELU)
        h2 = ops.linear(feat, W["fc2.weight"], W["fc2.bias"], act=ops.ACT_RELU)
        return h1, h2

    def heads(self, feat, want_pi=True, pi=None, v=None):
        """TicTacToeGNN.py:36-45."""
        W = self.params
        h1, h2 = self.hidden(feat)
        return ops.heads(h1, W["fc_policy.weight"], W["fc_policy.bias"], W["fc_value.weight"],
                         W["fc_value.bias"], hv=h2, want_pi=want_pi, pi=pi, v=v)

    def __call__(self, b):
        logp, _, v = self.heads(self.features(b), want_pi=False)
        return logp, v.view(-1, 1)


class GNNLayer:
    """gnn_utils.py:5-74 parameters of layer i as views into the parent's flat buffer."""

    def __init__(self, params, i):
        self.prefix = f"layers.{i}."
        self.params = params

    def weights(self):
        p = self.prefix
        return {k[len(p):]: v for k, v in self.params.views.items() if k.startswith(p)}


class PolicyValueGNN(_Net):
    """gnn_utils.py:87-117: `num_layers` GNNLayers then output_transform (Linear-ReLU-Linear)."""

    def __init__(self, feature_dim, num_layers=2, device=None, init=None):
        self.feature_dim = feature_dim
        self.num_layers = num_layers
        spec = gnn_spec(feature_dim, num_layers)
        self.params = FlatParams(spec, device or default_device(),
                                 init if init is not None else torch_default_init(spec))
        self.layers = [GNNLayer(self.params, i) for i in range(num_layers)]
        self.training = True
        self._graphs = {}
        self._ws = None

    def _star(self, n):
        g = self._graphs.get(n)
        if g is None:
            g = self._graphs[n] = ops.DeviceGraph.star(n, self.params.device)
        return g

    def output_transform(self, x):
        W = self.params
        W.sync()
        y, _ = ops.mlp2(x, W["output_transform.0.weight"], W["output_transform.0.bias"],
                        W["output_transform.2.weight"], W["output_transform.2.bias"])
        return y

    def run_layers(self, x, graph):
        """The layer stack; in eval mode nothing is kept for a backward pass
        (az_gnn_layer_infer: one fused kernel per layer on grid-shaped graphs)."""
        self.params.sync()
        for layer in self.layers:
            x, self._ws = ops.gnn_layer(graph, x, layer.weights(), ws=self._ws,
                                        save=self.training)
        return x

    def __call__(self, features):
        """Exactly the reference's forward: the whole input is ONE star (row 0 <- rows 1..N-1);
        a 1-row input passes the layers unchanged (gnn_utils.py:35-36)."""
        x = features
        if x.shape[0] > 1:
            x = self.run_layers(x, self._star(x.shape[0]))
        return self.output_transform(x)

    def forward_per_row(self, features):
        """Each row as its own 1-row input (batched predict_with_gnn semantics)."""
        return self.output_transform(features)

    def forward_graph(self, x, graph):
        """Per-destination generalisation over a CSR graph (synthetic grid workload).  In eval
        mode the last layer and output_transform are one call (az_gnn_layer_ot_infer: on band
        graphs one launch, the layer's output never reaches HBM)."""
        if self.training or not self.layers:
            return self.output_transform(self.run_layers(x, graph))
        self.params.sync()
        for layer in self.layers[:-1]:
            x, self._ws = ops.gnn_layer(graph, x, layer.weights(), ws=self._ws, save=False)
        W = self.params
        y, self._ws = ops.gnn_layer_ot(graph, x, self.layers[-1].weights(),
                                       W["output_transform.0.weight"],
                                       W["output_transform.0.bias"],
                                       W["output_transform.2.weight"],
                                       W["output_transform.2.bias"], ws=self._ws)
        return y


def gnn_per_row_heads(nnet, gnn, feat, want_pi=True, pi=None, v=None):
    """Batched predict_with_gnn after extract_features (Connect4GNN.py:108-114 applied per row:
    the layers are the identity on a 1-row input, gnn_utils.py:35-36) -> (logp, pi, v).
    Connect4 heads read the transform output directly, so the whole tail is one
    az_transform_heads_fwd call; TicTacToe's heads go through fc1/fc2 first."""
    if isinstance(nnet, Connect4Net):
        G, W = gnn.params, nnet.params
        G.sync()
        W.sync()
        logp, pi, v, _, _ = ops.transform_heads(
            feat, G["output_transform.0.weight"], G["output_transform.0.bias"],
            G["output_transform.2.weight"], G["output_transform.2.bias"], W["fc_policy.weight"],
            W["fc_policy.bias"], W["fc_value.weight"], W["fc_value.bias"], want_pi=want_pi,
            pi=pi, v=v, want_y=False)
        return logp, pi, v
    return nnet.heads(gnn.forward_per_row(feat), want_pi=want_pi, pi=pi, v=v)


class C4Evaluator:
    """Connect4 board evaluator from plain state dicts (bench / smoke convenience)."""

    def __init__(self, W, G=None, device=None, num_layers=2, n=7):
        device = device or default_device()
        game = SimpleNamespace(getBoardSize=lambda: (n, n), getActionSize=lambda: n + 1)
        self.nnet = Connect4Net(game, {"dropout": 0.0}, device=device, init=W).eval()
        self.gnn = (PolicyValueGNN(64 * n * n, num_layers, device=device, init=G).eval()
                    if G is not None else None)
        self.device = self.nnet.params.device

    def evaluate(self, b, gnn=False):
        """Device in, device out: int8 boards [B,n,n] -> (logp, pi, v) on HBM, no sync."""
        f = self.nnet.features(b)
        if gnn:
            return gnn_per_row_heads(self.nnet, self.gnn, f)
        return self.nnet.heads(f)

    def predict_batch(self, boards, gnn=False):
        b = boards_to_device(boards, self.device)
        _, pi, v = self.evaluate(b, gnn)
        return pi.cpu().numpy(), v.cpu().numpy()

    def star_forward(self, boards):
        b = boards_to_device(boards, self.device)
        logp, _, v = self.nnet.heads(self.gnn(self.nnet.features(b)), want_pi=False)
        return logp.cpu().numpy(), v.cpu().numpy()

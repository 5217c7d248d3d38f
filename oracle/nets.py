"""numpy restatement of the reference networks (ORACLE: test infrastructure only).

All functions take plain numpy arrays and a dict of weights keyed like the reference
``state_dict`` (``azhip.weights`` specs).  ``dtype`` selects the arithmetic: float64 for
parity checks (a tighter truth than the reference's own fp32), float32 for the CPU
baseline timing in bench.py.
"""
import numpy as np


def _w(W, k, dtype):
    return np.asarray(W[k], dtype=dtype)


def conv2d(x, w, b, pad):
    """nn.Conv2d(k=3, stride=1, padding=pad) on NCHW ``x`` (torch semantics: cross-correlation).
    Used by connect4/Connect4Net.py:45-46 and tictactoe/TicTacToeNet.py:33-35."""
    B, C, H, Wd = x.shape
    O, C2, kh, kw = w.shape
    assert C == C2
    if pad:
        x = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    Ho, Wo = x.shape[2] - kh + 1, x.shape[3] - kw + 1
    s = x.strides
    cols = np.lib.stride_tricks.as_strided(
        x, shape=(B, Ho, Wo, C, kh, kw), strides=(s[0], s[2], s[3], s[1], s[2], s[3]))
    cols = cols.reshape(B * Ho * Wo, C * kh * kw)
    y = cols @ w.reshape(O, -1).T + b
    return y.reshape(B, Ho, Wo, O).transpose(0, 3, 1, 2)


def relu(x):
    return np.maximum(x, 0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def log_softmax(x):
    m = x.max(axis=1, keepdims=True)
    z = x - m
    return z - np.log(np.exp(z).sum(axis=1, keepdims=True))


# ------------------------------------------------------------------------------ Connect4
def c4_features(boards, W, dtype=np.float64):
    """Connect4Net.forward trunk up to the flatten, connect4/Connect4Net.py:42-49
    (== Connect4GNNWrapper.extract_features, connect4/Connect4GNN.py:31-46, dropout off).
    boards: [B, n, n] in {-1,0,1} (axis 0 = column x -> conv H, axis 1 = row y -> conv W)."""
    B, n, _ = boards.shape
    s = np.asarray(boards, dtype=dtype).reshape(B, 1, n, n)
    s = relu(conv2d(s, _w(W, "conv1.weight", dtype), _w(W, "conv1.bias", dtype), 1))
    s = relu(conv2d(s, _w(W, "conv2.weight", dtype), _w(W, "conv2.bias", dtype), 1))
    return s.reshape(B, 64 * n * n)  # NCHW flatten: c*n*n + x*n + y


def c4_heads(feat, W, dtype=np.float64):
    """Connect4Net.py:54-60 / Connect4GNN.py:48-57: fc_policy -> log_softmax, fc_value -> tanh."""
    f = np.asarray(feat, dtype=dtype)
    pi = f @ _w(W, "fc_policy.weight", dtype).T + _w(W, "fc_policy.bias", dtype)
    v = np.tanh(f @ _w(W, "fc_value.weight", dtype).T + _w(W, "fc_value.bias", dtype))
    return log_softmax(pi), v[:, 0]


def c4_forward(boards, W, dtype=np.float64):
    """Connect4Net.forward in eval mode, connect4/Connect4Net.py:30-60."""
    return c4_heads(c4_features(boards, W, dtype), W, dtype)


# ------------------------------------------------------------------------------ TicTacToe
def ttt_features(boards, W, dtype=np.float64):
    """TicTacToeNet.forward trunk, tictactoe/TicTacToeNet.py:30-38 (conv3 has NO padding)."""
    B, n, _ = boards.shape
    s = np.asarray(boards, dtype=dtype).reshape(B, 1, n, n)
    s = relu(conv2d(s, _w(W, "conv1.weight", dtype), _w(W, "conv1.bias", dtype), 1))
    s = relu(conv2d(s, _w(W, "conv2.weight", dtype), _w(W, "conv2.bias", dtype), 1))
    s = relu(conv2d(s, _w(W, "conv3.weight", dtype), _w(W, "conv3.bias", dtype), 0))
    return s.reshape(B, 128 * (n - 2) * (n - 2))


def ttt_heads(feat, W, dtype=np.float64):
    """tictactoe/TicTacToeNet.py:40-48 (== TicTacToeGNN.py:36-45)."""
    f = np.asarray(feat, dtype=dtype)
    p = relu(f @ _w(W, "fc1.weight", dtype).T + _w(W, "fc1.bias", dtype))
    p = p @ _w(W, "fc_policy.weight", dtype).T + _w(W, "fc_policy.bias", dtype)
    v = relu(f @ _w(W, "fc2.weight", dtype).T + _w(W, "fc2.bias", dtype))
    v = np.tanh(v @ _w(W, "fc_value.weight", dtype).T + _w(W, "fc_value.bias", dtype))
    return log_softmax(p), v[:, 0]


def ttt_forward(boards, W, dtype=np.float64):
    return ttt_heads(ttt_features(boards, W, dtype), W, dtype)


# ------------------------------------------------------------------------------ GNN
def _layer(G, i, dtype):
    p = f"layers.{i}."
    return {k: _w(G, p + k, dtype) for k in (
        "attention.0.weight", "attention.0.bias", "attention.2.weight", "attention.2.bias",
        "update_net.0.weight", "update_net.0.bias", "update_net.2.weight", "update_net.2.bias",
        "gate.0.weight", "gate.0.bias")}


def attention_scores(t, src, L):
    """GNNLayer.compute_attention for each source, gnn_utils.py:30-32,48-55:
    sigma(w2 . relu(W1 [t; x_i] + b1) + b2); returns [n_src]."""
    comb = np.concatenate([np.broadcast_to(t, (src.shape[0], t.shape[1])), src], axis=1)
    h = relu(comb @ L["attention.0.weight"].T + L["attention.0.bias"])
    return sigmoid(h @ L["attention.2.weight"].T + L["attention.2.bias"])[:, 0]


def node_update(t, agg, L):
    """gnn_utils.py:67-71: c=[t;agg]; t + sigmoid(Wg c+bg) * (Wu2 relu(Wu1 c+bu1)+bu2)."""
    c = np.concatenate([t, agg], axis=1)
    g = sigmoid(c @ L["gate.0.weight"].T + L["gate.0.bias"])
    u = relu(c @ L["update_net.0.weight"].T + L["update_net.0.bias"])
    u = u @ L["update_net.2.weight"].T + L["update_net.2.bias"]
    return t + g * u


def gnn_layer_star(features, G, i, dtype=np.float64, trace=None):
    """GNNLayer.forward, gnn_utils.py:34-74.  Row 0 is the single destination, rows 1..N-1
    its sources; only row 0 changes.  ``trace`` (dict) receives alpha/agg when given."""
    x = np.asarray(features, dtype=dtype)
    if x.shape[0] <= 1:                                   # :35-36
        return x
    L = _layer(G, i, dtype)
    t, src = x[0:1], x[1:]
    a = attention_scores(t, src, L)                       # :48-55
    s = a.sum()
    if s > 0:                                             # :58-59
        a = a / s
    agg = (src * a[:, None]).sum(axis=0, keepdims=True)   # :62-65
    if trace is not None:
        trace.setdefault("alpha_raw", []).append(a * s if s > 0 else a)
        trace.setdefault("agg", []).append(agg[0])
    return np.concatenate([node_update(t, agg, L), src], axis=0)   # :68-74


def gnn_layer_csr(x, rowptr, col, G, i, dtype=np.float64):
    """Per-destination generalisation of GNNLayer (SURVEY.md §8 vocabulary map):
    x'[d] = GNNLayer(cat[x_d, x_N(d)])[0] for every destination d of a dst-sorted CSR.
    A destination with no in-edges is GNNLayer on a 1-row input: unchanged (gnn_utils.py:35)."""
    x = np.asarray(x, dtype=dtype)
    L = _layer(G, i, dtype)
    deg = np.diff(rowptr)
    dst = np.repeat(np.arange(len(deg)), deg)
    src = np.asarray(col)
    a = attention_scores_pairs(x[dst], x[src], L)
    ssum = np.zeros(len(deg), dtype)
    np.add.at(ssum, dst, a)
    w = np.where(ssum[dst] > 0, a / np.where(ssum[dst] > 0, ssum[dst], 1), a)
    agg = np.zeros_like(x)
    np.add.at(agg, dst, x[src] * w[:, None])
    out = x.copy()
    has = deg > 0
    out[has] = node_update(x[has], agg[has], L)
    return out


def attention_scores_pairs(t, s, L):
    comb = np.concatenate([t, s], axis=1)
    h = relu(comb @ L["attention.0.weight"].T + L["attention.0.bias"])
    return sigmoid(h @ L["attention.2.weight"].T + L["attention.2.bias"])[:, 0]


def output_transform(x, G, dtype=np.float64):
    """gnn_utils.py:101-105,115: Linear(F,F) -> ReLU -> Linear(F,F) on every row."""
    h = relu(x @ _w(G, "output_transform.0.weight", dtype).T + _w(G, "output_transform.0.bias", dtype))
    return h @ _w(G, "output_transform.2.weight", dtype).T + _w(G, "output_transform.2.bias", dtype)


def policy_value_gnn_star(features, G, num_layers=2, dtype=np.float64, trace=None):
    """PolicyValueGNN.forward, gnn_utils.py:107-117 (the star semantics of training)."""
    x = np.array(features, dtype=dtype)
    for i in range(num_layers):
        x = gnn_layer_star(x, G, i, dtype, trace)
    return output_transform(x, G, dtype)


def policy_value_gnn_per_row(features, G, dtype=np.float64):
    """predict_with_gnn semantics applied row by row (Connect4GNN.py:86-120): each board is a
    1-row input, so the layers are the identity (gnn_utils.py:35-36) -> output_transform only."""
    return output_transform(np.asarray(features, dtype=dtype), G, dtype)


def policy_value_gnn_csr(x, rowptr, col, G, num_layers=2, dtype=np.float64):
    for i in range(num_layers):
        x = gnn_layer_csr(x, rowptr, col, G, i, dtype)
    return output_transform(x, G, dtype)


# ------------------------------------------------------------------------------ losses / Adam
def losses(log_pi, v, target_pi, target_v):
    """Connect4GNN.py:150-152,187-193: -sum(pi*logp)/B and sum((z-v)^2)/B."""
    B = target_pi.shape[0]
    return -(target_pi * log_pi).sum() / B, ((target_v - v) ** 2).sum() / B


class Adam:
    """torch.optim.Adam defaults (betas (0.9, 0.999), eps 1e-8, no weight decay, no amsgrad),
    the algorithm the reference constructs fresh in every train() (Connect4GNN.py:132-133):
    m <- lerp(m, g, 1-b1); v <- b2 v + (1-b2) g^2; p <- p - (lr/bc1) m / (sqrt(v)/sqrt(bc2) + eps)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = {k: np.zeros_like(v) for k, v in params.items()}
        self.v = {k: np.zeros_like(v) for k, v in params.items()}
        self.t = 0

    def step(self, params, grads):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        for k in params:
            g = grads[k]
            self.m[k] = self.m[k] + (1 - self.b1) * (g - self.m[k])
            self.v[k] = self.v[k] * self.b2 + (1 - self.b2) * g * g
            denom = np.sqrt(self.v[k]) / np.sqrt(bc2) + self.eps
            params[k] = params[k] - (self.lr / bc1) * self.m[k] / denom
        return params

"""torch-CPU restatement of the reference forward pass with autograd (ORACLE: test
infrastructure only).  Used as the fp64 gradient reference for the HIP backward kernels;
the numpy restatement in oracle/nets.py is the forward oracle.  Functional form, weights
passed as dicts keyed like the reference state_dict."""
import torch
import torch.nn.functional as F


def params(sd, dtype=torch.float64, requires_grad=True):
    out = {}
    for k, v in sd.items():
        t = torch.as_tensor(v).detach().to(dtype).clone()
        t.requires_grad_(requires_grad)
        out[k] = t
    return out


def c4_features(boards, W, drop_mask=None, p=0.0):
    """connect4/Connect4Net.py:42-52 (dropout as an explicit keep-mask, F.dropout scaling)."""
    B, n, _ = boards.shape
    s = torch.as_tensor(boards).to(W["conv1.weight"].dtype).view(B, 1, n, n)
    s = F.relu(F.conv2d(s, W["conv1.weight"], W["conv1.bias"], padding=1))
    s = F.relu(F.conv2d(s, W["conv2.weight"], W["conv2.bias"], padding=1))
    s = s.reshape(B, -1)
    if drop_mask is not None:
        s = s * torch.as_tensor(drop_mask).to(s.dtype).view_as(s) / (1.0 - p)
    return s


def c4_heads(f, W):
    """Connect4GNN.py:48-57."""
    pi = F.linear(f, W["fc_policy.weight"], W["fc_policy.bias"])
    v = torch.tanh(F.linear(f, W["fc_value.weight"], W["fc_value.bias"]))
    return F.log_softmax(pi, dim=1), v.view(-1)


def ttt_features(boards, W):
    """tictactoe/TicTacToeNet.py:30-38."""
    B, n, _ = boards.shape
    s = torch.as_tensor(boards).to(W["conv1.weight"].dtype).view(B, 1, n, n)
    s = F.relu(F.conv2d(s, W["conv1.weight"], W["conv1.bias"], padding=1))
    s = F.relu(F.conv2d(s, W["conv2.weight"], W["conv2.bias"], padding=1))
    s = F.relu(F.conv2d(s, W["conv3.weight"], W["conv3.bias"]))
    return s.reshape(B, -1)


def ttt_heads(f, W):
    """tictactoe/TicTacToeNet.py:40-48."""
    p = F.linear(F.relu(F.linear(f, W["fc1.weight"], W["fc1.bias"])), W["fc_policy.weight"],
                 W["fc_policy.bias"])
    v = F.linear(F.relu(F.linear(f, W["fc2.weight"], W["fc2.bias"])), W["fc_value.weight"],
                 W["fc_value.bias"])
    return F.log_softmax(p, dim=1), torch.tanh(v).view(-1)


def losses(logp, v, tpi, tv):
    """Connect4GNN.py:150-152 / :187-193."""
    tpi = torch.as_tensor(tpi).to(logp.dtype)
    tv = torch.as_tensor(tv).to(logp.dtype)
    B = tpi.shape[0]
    return -(tpi * logp).sum() / B + ((tv - v) ** 2).sum() / B


def _L(G, i):
    p = f"layers.{i}."
    return {k[len(p):]: v for k, v in G.items() if k.startswith(p)}


def gnn_layer_csr(x, rowptr, col, G, i):
    """Per-destination GNNLayer (gnn_utils.py:34-74): x'[d] = GNNLayer(cat[x_d, x_N(d)])[0];
    destinations without in-edges pass through (:35-36).  Vectorised over edges."""
    L = _L(G, i)
    rowptr = torch.as_tensor(rowptr, dtype=torch.long)
    col = torch.as_tensor(col, dtype=torch.long)
    V = x.shape[0]
    deg = rowptr[1:] - rowptr[:-1]
    dst = torch.repeat_interleave(torch.arange(V), deg)
    comb = torch.cat([x[dst], x[col]], dim=1)
    h = F.relu(F.linear(comb, L["attention.0.weight"], L["attention.0.bias"]))
    a = torch.sigmoid(F.linear(h, L["attention.2.weight"], L["attention.2.bias"]))[:, 0]
    S = torch.zeros(V, dtype=x.dtype).index_add(0, dst, a)
    w = torch.where(S[dst] > 0, a / torch.where(S[dst] > 0, S[dst], torch.ones_like(a)), a)
    agg = torch.zeros_like(x).index_add(0, dst, x[col] * w[:, None])
    c = torch.cat([x, agg], dim=1)
    g = torch.sigmoid(F.linear(c, L["gate.0.weight"], L["gate.0.bias"]))
    u = F.linear(F.relu(F.linear(c, L["update_net.0.weight"], L["update_net.0.bias"])),
                 L["update_net.2.weight"], L["update_net.2.bias"])
    upd = x + g * u
    has = (deg > 0)[:, None]
    return torch.where(has, upd, x)


def star_csr(n):
    rowptr = [0] + [n - 1] * n
    return rowptr, list(range(1, n))


def output_transform(x, G):
    """gnn_utils.py:101-105,115."""
    h = F.relu(F.linear(x, G["output_transform.0.weight"], G["output_transform.0.bias"]))
    return F.linear(h, G["output_transform.2.weight"], G["output_transform.2.bias"])


def policy_value_gnn(x, G, num_layers=2, rowptr=None, col=None):
    """gnn_utils.py:107-117; the default graph is the reference's star over the rows."""
    if rowptr is None:
        rowptr, col = star_csr(x.shape[0])
    for i in range(num_layers):
        x = gnn_layer_csr(x, rowptr, col, G, i)
    return output_transform(x, G)

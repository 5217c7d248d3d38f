"""Training steps of the reference's NeuralNet.train on libaz_hip (no autograd: explicit HIP
backward kernels + a fused Adam over the flat parameter buffer).

* cnn_step  -- Connect4Net / TicTacToeNet step: Connect4GNN.py:140-156, TicTacToeGNN.py:206-223
* gnn_step  -- the GNN step on the star over the sampled batch: Connect4GNN.py:159-197.
               Only PolicyValueGNN parameters are updated there; the reference's backward also
               writes .grad of the conv trunk / heads, but the next epoch's
               nnet_optimizer.zero_grad() (Connect4GNN.py:154) discards them unused, so that
               dead work is skipped.

Every step takes device tensors: boards int8 [B,n,n], target pi fp32 [B,A], target v fp32 [B].
"""
import torch

from . import ops


def _views(net):
    return net.params.views


def _grads(net):
    net.params.grad_flat  # allocate
    return net.params.grads


def adam_step(net, lr):
    P = net.params
    P.step += 1
    ops.adam(P.flat, P.grad_flat, P.m, P.v, lr, P.step)


# ------------------------------------------------------------------------------ features
class C4Forward:
    """Connect4Net forward in train mode keeping what the backward needs."""

    def __init__(self, net, boards, drop_p=0.0, seed=0, mask=None):
        W = _views(net)
        self.boards = boards
        self.B = boards.shape[0]
        self.n = net.n
        self.feat = net.features(boards)                         # a2 = relu(conv2), NCHW flat
        self.p = float(drop_p)
        self.mask = mask
        if self.p > 0.0 and self.mask is None:
            self.mask = ops.dropout_mask(self.feat.numel(), self.p, seed, self.feat.device)
        self.scale = 1.0 / (1.0 - self.p) if self.p > 0.0 else 1.0
        self.s = (ops.mask_scale(self.feat, self.mask, self.scale) if self.mask is not None
                  else self.feat)
        self.W = W

    def trunk_backward(self, ds, G):
        """ds: d loss / d (dropped features) [B, 64*n*n] -> conv grads into G."""
        W, B, n = self.W, self.B, self.n
        HW = n * n
        dz2 = ops.nchw_drelu_to_pm(ds, self.feat, B, 64, HW, mask=self.mask, scale=self.scale)
        a1 = ops.conv3x3_relu(self.boards, W["conv1.weight"], W["conv1.bias"], 1)
        cols2 = ops.im2col3x3(a1, 1)                                          # [B*HW, 288]
        ops.matmul_tn(dz2, cols2, G["conv2.weight"].view(64, 288), 64, 288, B * HW)
        ops.colsum(dz2, G["conv2.bias"])
        dcols2 = torch.empty((B * HW, 288), device=ds.device)
        ops.matmul_nn(dz2, W["conv2.weight"].view(64, 288), dcols2, B * HW, 288, 64)
        dz1 = ops.col2im3x3_drelu(dcols2, a1, 1)                              # [B*HW, 32]
        cols1 = ops.im2col3x3(self.boards, 1)                                 # [B*HW, 12]
        ops.matmul_tn(dz1, cols1, G["conv1.weight"].view(32, 9), 32, 9, B * HW)
        ops.colsum(dz1, G["conv1.bias"])


class TTTForward:
    """TicTacToeNet forward (no dropout anywhere, TicTacToeNet.py:28-48) keeping activations."""

    def __init__(self, net, boards):
        W = _views(net)
        self.W, self.boards, self.B, self.n = W, boards, boards.shape[0], net.n
        self.a1 = ops.conv3x3_relu(boards, W["conv1.weight"], W["conv1.bias"], 1)
        self.a2 = ops.conv3x3_relu(self.a1, W["conv2.weight"], W["conv2.bias"], 1)
        self.a3 = ops.conv3x3_relu(self.a2, W["conv3.weight"], W["conv3.bias"], 0)
        self.s = self.a3.view(self.B, -1)

    def trunk_backward(self, ds, G):
        W, B, n = self.W, self.B, self.n
        m = n - 2
        dz3 = ops.nchw_drelu_to_pm(ds, self.a3, B, 128, m * m)
        cols3 = ops.im2col3x3(self.a2, 0)                                     # [B*m*m, 576]
        ops.matmul_tn(dz3, cols3, G["conv3.weight"].view(128, 576), 128, 576, B * m * m)
        ops.colsum(dz3, G["conv3.bias"])
        dcols3 = torch.empty((B * m * m, 576), device=ds.device)
        ops.matmul_nn(dz3, W["conv3.weight"].view(128, 576), dcols3, B * m * m, 576, 128)
        dz2 = ops.col2im3x3_drelu(dcols3, self.a2, 0)                         # [B*n*n, 64]
        cols2 = ops.im2col3x3(self.a1, 1)
        ops.matmul_tn(dz2, cols2, G["conv2.weight"].view(64, 288), 64, 288, B * n * n)
        ops.colsum(dz2, G["conv2.bias"])
        dcols2 = torch.empty((B * n * n, 288), device=ds.device)
        ops.matmul_nn(dz2, W["conv2.weight"].view(64, 288), dcols2, B * n * n, 288, 64)
        dz1 = ops.col2im3x3_drelu(dcols2, self.a1, 1)
        cols1 = ops.im2col3x3(self.boards, 1)
        ops.matmul_tn(dz1, cols1, G["conv1.weight"].view(32, 9), 32, 9, B * n * n)
        ops.colsum(dz1, G["conv1.bias"])


# ------------------------------------------------------------------------------ heads
def c4_heads_fwd(net, s):
    W = _views(net)
    logp, _, v = ops.heads(s, W["fc_policy.weight"], W["fc_policy.bias"], W["fc_value.weight"],
                           W["fc_value.bias"], want_pi=False)
    return logp, v, None


def c4_heads_bwd(net, s, dl, dv, saved, G=None):
    """Returns d loss / d s; writes fc grads into G when given."""
    W = _views(net)
    ds = torch.empty_like(s)
    grads = None
    if G is not None:
        grads = {"wp": G["fc_policy.weight"], "bp": G["fc_policy.bias"],
                 "wv": G["fc_value.weight"], "bv": G["fc_value.bias"]}
    ops.heads_bwd(dl, dv, s, W["fc_policy.weight"], W["fc_value.weight"], grads=grads, dh=ds)
    return ds


def ttt_heads_fwd(net, s):
    W = _views(net)
    h1 = ops.linear(s, W["fc1.weight"], W["fc1.bias"], act=ops.ACT_RELU)
    h2 = ops.linear(s, W["fc2.weight"], W["fc2.bias"], act=ops.ACT_RELU)
    logp, _, v = ops.heads(h1, W["fc_policy.weight"], W["fc_policy.bias"], W["fc_value.weight"],
                           W["fc_value.bias"], hv=h2, want_pi=False)
    return logp, v, (h1, h2)


def ttt_heads_bwd(net, s, dl, dv, saved, G=None):
    W = _views(net)
    h1, h2 = saved
    B = s.shape[0]
    dh1, dh2 = torch.empty_like(h1), torch.empty_like(h2)
    grads = None
    if G is not None:
        grads = {"wp": G["fc_policy.weight"], "bp": G["fc_policy.bias"],
                 "wv": G["fc_value.weight"], "bv": G["fc_value.bias"]}
    ops.heads_bwd(dl, dv, h1, W["fc_policy.weight"], W["fc_value.weight"], hv=h2, grads=grads,
                  dh=dh1, dhv=dh2)
    d1 = ops.nchw_drelu_to_pm(dh1, h1, B, h1.shape[1], 1)       # relu backward (layout no-op)
    d2 = ops.nchw_drelu_to_pm(dh2, h2, B, h2.shape[1], 1)
    K = s.shape[1]
    if G is not None:
        ops.matmul_tn(d1, s, G["fc1.weight"], 512, K, B)
        ops.colsum(d1, G["fc1.bias"])
        ops.matmul_tn(d2, s, G["fc2.weight"], 512, K, B)
        ops.colsum(d2, G["fc2.bias"])
    ds = torch.empty_like(s)
    ops.matmul_nn(d1, W["fc1.weight"], ds, B, K, 512)
    ops.matmul_nn(d2, W["fc2.weight"], ds, B, K, 512, beta=1.0)
    return ds


def _kind(net):
    return "c4" if hasattr(net, "dropout") else "ttt"


# ------------------------------------------------------------------------------ steps
def cnn_grads(net, boards, tpi, tv, seed=0, drop_mask=None, B_norm=None):
    """Forward in train mode, loss -sum(pi*logp)/B + sum((z-v)^2)/B (Connect4GNN.py:148-152)
    and its gradient into net.params.grads.  Returns (l_pi, l_v) on the device."""
    G = _grads(net)
    if _kind(net) == "c4":
        fw = C4Forward(net, boards, net.dropout, seed, drop_mask)
        logp, v, saved = c4_heads_fwd(net, fw.s)
    else:
        fw = TTTForward(net, boards)
        logp, v, saved = ttt_heads_fwd(net, fw.s)
    lrows = torch.empty((boards.shape[0], 2), device=boards.device)
    dl, dv = ops.heads_loss_bwd(logp, v, tpi, tv, B_norm=B_norm, loss_rows=lrows)
    if _kind(net) == "c4":
        ds = c4_heads_bwd(net, fw.s, dl, dv, saved, G)
    else:
        ds = ttt_heads_bwd(net, fw.s, dl, dv, saved, G)
    fw.trunk_backward(ds, G)
    return lrows.sum(0)


def cnn_step(net, boards, tpi, tv, lr, seed=0, drop_mask=None, B_norm=None):
    """One reference CNN training step (Connect4GNN.py:141-156): grads then Adam."""
    loss = cnn_grads(net, boards, tpi, tv, seed, drop_mask, B_norm)
    adam_step(net, lr)
    return loss


class GNNForward:
    """extract_features -> PolicyValueGNN (star over the rows) -> heads, keeping activations."""

    def __init__(self, net, gnn, boards, seed=0, drop_mask=None):
        self.net, self.gnn = net, gnn
        if _kind(net) == "c4":
            fw = C4Forward(net, boards, net.dropout, seed, drop_mask)   # Connect4GNN.py:44
        else:
            fw = TTTForward(net, boards)
        x = fw.s.contiguous()
        self.xs = [x]
        self.ws = []
        self.graph = gnn._star(x.shape[0]) if x.shape[0] > 1 else None
        if self.graph is not None:
            for layer in gnn.layers:
                x, ws = ops.gnn_layer(self.graph, x, layer.weights())
                self.xs.append(x)
                self.ws.append(ws)
        Wg = gnn.params.views
        self.y, self.hidden = ops.mlp2(x, Wg["output_transform.0.weight"],
                                       Wg["output_transform.0.bias"],
                                       Wg["output_transform.2.weight"],
                                       Wg["output_transform.2.bias"])
        if _kind(net) == "c4":
            self.logp, self.v, self.saved = c4_heads_fwd(net, self.y)
        else:
            self.logp, self.v, self.saved = ttt_heads_fwd(net, self.y)

    def backward(self, dl, dv, GG):
        net, gnn = self.net, self.gnn
        if _kind(net) == "c4":
            dy = c4_heads_bwd(net, self.y, dl, dv, self.saved, None)
        else:
            dy = ttt_heads_bwd(net, self.y, dl, dv, self.saved, None)
        Wg = gnn.params.views
        xl = self.xs[-1]
        dx = ops.mlp2_bwd(xl, Wg["output_transform.0.weight"], Wg["output_transform.2.weight"],
                          self.hidden, dy,
                          {"w0": GG["output_transform.0.weight"],
                           "b0": GG["output_transform.0.bias"],
                           "w2": GG["output_transform.2.weight"],
                           "b2": GG["output_transform.2.bias"]},
                          want_dx=self.graph is not None)
        if self.graph is None:
            for layer in gnn.layers:                     # 1-row input: layers are the identity
                for k, g in GG.items():
                    if k.startswith(layer.prefix):
                        g.zero_()
            return
        for li in range(len(gnn.layers) - 1, -1, -1):
            layer = gnn.layers[li]
            grads = {k[len(layer.prefix):]: v for k, v in GG.items() if k.startswith(layer.prefix)}
            dx = ops.gnn_layer_bwd(self.graph, self.xs[li], layer.weights(), self.ws[li], dx,
                                   grads)


def gnn_grads(net, gnn, boards, tpi, tv, seed=0, drop_mask=None):
    """GNN-step loss (Connect4GNN.py:187-193) and its gradient w.r.t. the GNN parameters."""
    GG = _grads(gnn)
    fw = GNNForward(net, gnn, boards, seed, drop_mask)
    lrows = torch.empty((boards.shape[0], 2), device=boards.device)
    dl, dv = ops.heads_loss_bwd(fw.logp, fw.v, tpi, tv, loss_rows=lrows)
    fw.backward(dl, dv, GG)
    return lrows.sum(0)


def gnn_step(net, gnn, boards, tpi, tv, lr, seed=0, drop_mask=None):
    """One reference GNN training step (Connect4GNN.py:160-197) on the star over the batch."""
    loss = gnn_grads(net, gnn, boards, tpi, tv, seed, drop_mask)
    adam_step(gnn, lr)
    return loss


# ------------------------------------------------------------------------------ data parallel
def gnn_grads_dp(net, gnn, boards, tpi, tv, seed=0, grad_sync="row0"):
    """The GNN step's gradient, data parallel over the ranks.  `boards`, `tpi`,
    `tv` are the GLOBAL sampled batch (identical on every rank: the host RNGs are synchronised).

    The batch is ONE star: row 0 aggregates every other row, and only row 0's path reaches the
    layer parameters (gnn_utils.py:34-74; rows 1.. pass through unchanged).  So:
      1. the conv trunk runs on this rank's rows only (row_shard), with the global batch's
         dropout mask sliced to them (Connect4GNN.py:178 -> extract_features, dropout on);
      2. the features are gathered ([B, F], 800 KB at B = 64, F = 3136);
      3. every rank runs the star's layer stack (row 0 changes; rows 1.. are copies);
      4. output_transform, heads and the loss run on this rank's rows, normalised by the global
         B (Connect4GNN.py:187-193), giving output_transform's gradient over these rows;
      5. d loss / d x_L[0] lives on row 0's owner (rank 0).  grad_sync "row0": it is broadcast
         (12.5 KB) and every rank back-propagates the layer stack from it -- identical,
         deterministic kernels, so identical layer gradients -- and only output_transform's
         span of the flat gradient is all-reduced; "flat": only rank 0 back-propagates the
         layers, the other ranks' layer gradients are zero, and the whole flat gradient is
         all-reduced in one bucket (the literal §8e exchange).
    The conv-trunk backward stays skipped (dead work, see gnn_step).  Returns (l_pi, l_v) summed
    over ALL rows (each rank's own-row partial sums all-reduced)."""
    from . import dist as D
    world, rank = D.world_rank()
    B = boards.shape[0]
    r0, r1 = D.row_shard(B, world, rank)
    GG = _grads(gnn)
    F = net.feature_dim
    if _kind(net) == "c4":
        drop = float(net.dropout)
        mask = ops.dropout_mask(B * F, drop, seed, boards.device) if drop > 0.0 else None
        own = (C4Forward(net, boards[r0:r1], drop, seed, None if mask is None else
                         mask[r0 * F:r1 * F]).s if r1 > r0
               else torch.empty((0, F), device=boards.device))
    else:
        own = (TTTForward(net, boards[r0:r1]).s if r1 > r0
               else torch.empty((0, F), device=boards.device))
    x = D.gather_rows(own.contiguous(), B, world, rank)
    xs, wss = [x], []
    graph = gnn._star(B) if B > 1 else None
    if graph is not None:
        for layer in gnn.layers:
            x, ws = ops.gnn_layer(graph, x, layer.weights())
            xs.append(x)
            wss.append(ws)
    Wg = gnn.params.views
    P = gnn.params
    GG["output_transform.0.weight"].zero_()          # a rank without rows contributes zeros
    GG["output_transform.0.bias"].zero_()
    GG["output_transform.2.weight"].zero_()
    GG["output_transform.2.bias"].zero_()
    lrows = torch.zeros((B, 2), device=boards.device)
    d0 = torch.zeros((1, F), device=boards.device)
    if r1 > r0:
        xo = xs[-1][r0:r1].contiguous()
        y, hidden = ops.mlp2(xo, Wg["output_transform.0.weight"], Wg["output_transform.0.bias"],
                             Wg["output_transform.2.weight"], Wg["output_transform.2.bias"])
        if _kind(net) == "c4":
            logp, v, saved = c4_heads_fwd(net, y)
        else:
            logp, v, saved = ttt_heads_fwd(net, y)
        dl, dv = ops.heads_loss_bwd(logp, v, tpi[r0:r1], tv[r0:r1], B_norm=B,
                                    loss_rows=lrows[r0:r1])
        dy = (c4_heads_bwd if _kind(net) == "c4" else ttt_heads_bwd)(net, y, dl, dv, saved, None)
        own_row0 = r0 == 0 and graph is not None
        dxo = ops.mlp2_bwd(xo, Wg["output_transform.0.weight"], Wg["output_transform.2.weight"],
                           hidden, dy, {"w0": GG["output_transform.0.weight"],
                                        "b0": GG["output_transform.0.bias"],
                                        "w2": GG["output_transform.2.weight"],
                                        "b2": GG["output_transform.2.bias"]},
                           want_dx=own_row0)
        if own_row0:
            d0.copy_(dxo[0:1])
    layer_span = (0, P.span("output_transform.")[0])
    if graph is None:
        GG_flat = P.grad_flat
        GG_flat[layer_span[0]:layer_span[1]].zero_()  # 1-row input: the layers are the identity
    else:
        run_layers = True
        if grad_sync == "row0":
            D.broadcast_(d0, src=0)
        elif grad_sync == "flat":
            run_layers = rank == 0
        else:
            raise ValueError(f"grad_sync must be 'row0' or 'flat', not {grad_sync!r}")
        if run_layers:
            dx = torch.zeros_like(xs[-1])
            dx[0:1] = d0                             # only row 0 reaches the layer parameters
            for li in range(len(gnn.layers) - 1, -1, -1):
                layer = gnn.layers[li]
                grads = {k[len(layer.prefix):]: g for k, g in GG.items()
                         if k.startswith(layer.prefix)}
                dx = ops.gnn_layer_bwd(graph, xs[li], layer.weights(), wss[li], dx, grads)
        else:
            P.grad_flat[layer_span[0]:layer_span[1]].zero_()
    if grad_sync == "flat":
        D.allreduce_sum_(P.grad_flat)
    else:
        s, e = P.span("output_transform.")
        D.allreduce_sum_(P.grad_flat[s:e])
    D.allreduce_sum_(lrows)
    return lrows.sum(0)


def gnn_step_dp(net, gnn, boards, tpi, tv, lr, seed=0, grad_sync="row0"):
    """gnn_step, data parallel (gnn_grads_dp) then the identical Adam step on every rank."""
    loss = gnn_grads_dp(net, gnn, boards, tpi, tv, seed, grad_sync)
    adam_step(gnn, lr)
    return loss

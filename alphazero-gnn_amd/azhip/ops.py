"""Tensor-level wrappers over the C-ABI.  Tensors are torch CUDA(HIP) tensors used purely as
device memory; every FLOP runs in libaz_hip.so on the current torch stream."""
import contextlib
import ctypes

import torch

from . import _lib
from ._lib import (ACT_DRELU, ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH, GemmDesc, Graph,  # noqa: F401
                   LayerGrads, LayerW)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev(t):
    """Device for the outputs of an op whose input is `t` (a HostBuffer view -> current GPU)."""
    return t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())


def _need(t, dtype=torch.float32, name="tensor"):
    if t is None:
        return
    if not t.is_cuda and not _zero_copy(t):
        raise ValueError(f"{name} must live on the GPU (got {t.device})")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")


_ZC_RANGES = {}   # start address -> end of each live HostBuffer


def _zero_copy(t):
    """True when CPU tensor `t` lies inside a HostBuffer (device-mapped host memory)."""
    a = t.data_ptr()
    return any(s <= a < e for s, e in _ZC_RANGES.items())


class HostBuffer:
    """Zero-copy host staging (az_host_alloc): fine-grained pinned host memory the kernels read
    and write in place, exposed as CPU tensors.  The ops accept views of it wherever they take
    a device input or output, so a batch-1 evaluation needs no copy launches: the host writes
    the board, the graph runs, and after the stream synchronises the host reads the outputs."""

    def __init__(self, nbytes):
        L = _lib.lib()
        p = L.az_host_alloc(nbytes)
        if not p:
            raise RuntimeError(f"az_host_alloc: {L.az_last_error().decode()}")
        self.ptr, self.nbytes = int(p), int(nbytes)
        self._arr = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        self.bytes = torch.frombuffer(self._arr, dtype=torch.uint8)
        _ZC_RANGES[self.ptr] = self.ptr + self.nbytes

    def view(self, offset, dtype, shape):
        """CPU tensor of `shape` over bytes [offset, offset + its size) of the buffer."""
        n = torch.Size(shape).numel() * torch.empty((), dtype=dtype).element_size()
        if offset % 16 or offset + n > self.nbytes:
            raise ValueError("HostBuffer.view: misaligned or out of range")
        return self.bytes[offset:offset + n].view(dtype).view(shape)

    def close(self):
        if self.ptr:
            _ZC_RANGES.pop(self.ptr, None)
            self.bytes = self._arr = None
            _lib.lib().az_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown
            pass


_WS = {}
_WS_PINNED = {}


def workspace(device, nbytes=256 << 20):
    """Per-device split-K workspace (kept for the process lifetime; grows on demand, which
    frees the previous buffer -- so a captured hipGraph must not reference it: see
    `pinned_workspace`)."""
    key = str(device)
    t = _WS_PINNED.get(key)
    if t is not None:
        return t
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = _WS[key] = torch.empty((nbytes,), dtype=torch.uint8, device=device)
    return t


@contextlib.contextmanager
def pinned_workspace(device, t):
    """Every op on `device` uses the caller-owned workspace `t` inside the block (a graph
    capture keeps `t` alive with the graph, so its kernels never point at a buffer the growing
    shared workspace has freed).  The entry points check that it is large enough."""
    key = str(device)
    prev = _WS_PINNED.get(key)
    _WS_PINNED[key] = t
    try:
        yield t
    finally:
        if prev is None:
            _WS_PINNED.pop(key, None)
        else:
            _WS_PINNED[key] = prev


def _p2_bytes(d):
    """Workspace the fp16-form GEMM on pre-split planes (az_gemm.hip, P2) needs beyond the
    default for a large K-major GEMM: A's two fp16 planes [2][M][K] + row scales (0 otherwise)."""
    if (d.K >= 1024 and d.N >= 256 and d.K % 32 == 0 and d.a_kmajor and d.b_kmajor
            and not d.A2 and not d.a_rows):
        return 4 * d.M * d.K + 8 * (d.M + d.N) + (1 << 20)
    return 0


def gemm(desc, device=None):
    L = _lib.lib()
    if device is not None and not desc.ws:
        # large M (65,536 x 3136: 0.8 GB of A planes) gets room for the pre-split operands
        ws = workspace(device, max(256 << 20, _p2_bytes(desc)))
        desc.ws, desc.ws_bytes = ws.data_ptr(), ws.numel()
    _lib.check(L.az_gemm_f32(ctypes.byref(desc), _stream()), "az_gemm_f32")


def linear(x, w, b=None, act=ACT_NONE, out=None, x2=None, a_rows=None, R=None, G=None,
           c_rows=None, beta=0.0, M=None, C2=None):
    """out = act(cat(x, x2) @ w.T + b) (optionally gated residual R + G*(...)), nn.Linear layout.
    x: [M, K1] (row stride taken from the tensor), x2: [M, K2] or None, w: [N, K1+K2].
    Large GEMMs cache w's per-row fp16-form scales and planes when w lies in registered
    parameter storage (FlatParams registers its buffer; az_weights_register): after writing new
    values into it, call params.weights_changed() (include/az_hip.h az_weights_changed).  Other
    weights get per-call scales."""
    _need(x, name="x")
    _need(w, name="w")
    K1 = x.shape[1]
    K = K1 + (x2.shape[1] if x2 is not None else 0)
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"linear: w {tuple(w.shape)} vs K={K}")
    if M is None:
        M = a_rows.numel() if a_rows is not None else x.shape[0]
    if out is None:
        out = torch.empty((M, N), device=x.device, dtype=torch.float32)
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = x.data_ptr(), x.stride(0), 1
    if x2 is not None:
        d.A2, d.lda2, d.K0 = x2.data_ptr(), x2.stride(0), K1
    d.a_rows = a_rows.data_ptr() if a_rows is not None else None
    d.B, d.ldb, d.b_kmajor = w.data_ptr(), w.stride(0), 1
    d.bias = b.data_ptr() if b is not None else None
    d.act = act
    if R is not None:
        d.R, d.ldr = R.data_ptr(), R.stride(0)
    if G is not None:
        d.G, d.ldg = G.data_ptr(), G.stride(0)
    d.beta = beta
    d.C, d.ldc = out.data_ptr(), out.stride(0)
    d.c_rows = c_rows.data_ptr() if c_rows is not None else None
    if C2 is not None:
        d.C2, d.ldc2 = C2.data_ptr(), C2.stride(0)
    gemm(d, x.device)
    return out


def matmul_tn(a, b, out, M, N, K, beta=0.0, lda=None, ldb=None):
    """out[M,N] (+)= a^T b with a stored [K][M] and b stored [K][N] (weight gradients)."""
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = a.data_ptr(), lda or a.stride(0), 0
    d.B, d.ldb, d.b_kmajor = b.data_ptr(), ldb or b.stride(0), 0
    d.beta = beta
    d.C, d.ldc = out.data_ptr(), out.stride(0)
    gemm(d, out.device)
    return out


def matmul_nn(a, b, out, M, N, K, beta=0.0):
    """out[M,N] (+)= a[M,K] @ b[K,N] (input gradients: dX = dY @ W)."""
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = a.data_ptr(), a.stride(0), 1
    d.B, d.ldb, d.b_kmajor = b.data_ptr(), b.stride(0), 0
    d.beta = beta
    d.C, d.ldc = out.data_ptr(), out.stride(0)
    gemm(d, out.device)
    return out


def c4_trunk(boards_i8, W, out=None):
    """Connect4Net trunk (Connect4Net.py:42-49) on int8 boards [B,7,7] -> features [B,3136]."""
    _need(boards_i8, torch.int8, "boards")
    B = boards_i8.shape[0]
    if out is None:
        out = torch.empty((B, 3136), device=_dev(boards_i8), dtype=torch.float32)
    L = _lib.lib()
    _lib.check(L.az_c4_trunk_fwd(_p(boards_i8), B, _p(W["conv1.weight"]), _p(W["conv1.bias"]),
                                 _p(W["conv2.weight"]), _p(W["conv2.bias"]), _p(out), _stream()),
               "az_c4_trunk_fwd")
    return out


def c4_trunk_heads(boards_i8, W, feat=None, logp=None, pi=None, v=None, want_pi=True):
    """Trunk + policy/value heads (Connect4Net.py:42-60) -> (feat, logp, pi, v); one launch
    for B <= 320, bit-identical to c4_trunk then heads."""
    _need(boards_i8, torch.int8, "boards")
    B = boards_i8.shape[0]
    dev = _dev(boards_i8)
    A = W["fc_policy.weight"].shape[0]
    feat = torch.empty((B, 3136), device=dev) if feat is None else feat
    logp = torch.empty((B, A), device=dev) if logp is None else logp
    pi = (torch.empty((B, A), device=dev) if pi is None else pi) if want_pi else None
    v = torch.empty((B,), device=dev) if v is None else v
    L = _lib.lib()
    ws = workspace(dev, max(int(L.az_heads_ws_bytes(B, 3136, A)), 64 << 20))
    _lib.check(L.az_c4_trunk_heads_fwd(
        _p(boards_i8), B, _p(W["conv1.weight"]), _p(W["conv1.bias"]), _p(W["conv2.weight"]),
        _p(W["conv2.bias"]), _p(W["fc_policy.weight"]), _p(W["fc_policy.bias"]), A,
        _p(W["fc_value.weight"]), _p(W["fc_value.bias"]), _p(feat), _p(logp), _p(pi), _p(v),
        _p(ws), ctypes.c_size_t(ws.numel()), _stream()), "az_c4_trunk_heads_fwd")
    return feat, logp, pi, v


def conv3x3_relu(x, w, b, pad, out=None):
    """x: int8 [B,H,W] (Cin=1) or fp32 [B,Cin,H,W] -> fp32 [B,Cout,Ho,Wo]."""
    is_i8 = x.dtype == torch.int8
    if is_i8:
        _need(x, torch.int8, "x")
        B, H, Wd = x.shape
        Cin = 1
    else:
        _need(x, name="x")
        B, Cin, H, Wd = x.shape
    Cout = w.shape[0]
    Ho, Wo = H + 2 * pad - 2, Wd + 2 * pad - 2
    if out is None:
        out = torch.empty((B, Cout, Ho, Wo), device=_dev(x), dtype=torch.float32)
    L = _lib.lib()
    _lib.check(L.az_conv3x3_relu_fwd(_p(x), int(is_i8), B, Cin, H, Wd, _p(w), _p(b), Cout, pad,
                                     _p(out), _stream()), "az_conv3x3_relu_fwd")
    return out


def heads(hp, wp, bp, wv, bv, hv=None, want_pi=True, logp=None, pi=None, v=None):
    """logp = log_softmax(hp wp^T + bp); v = tanh(hv wv^T + bv) (hv defaults to hp)."""
    hv = hp if hv is None else hv
    B, K = hp.shape
    A = wp.shape[0]
    dev = hp.device
    logp = torch.empty((B, A), device=dev) if logp is None else logp
    pi = (torch.empty((B, A), device=dev) if pi is None else pi) if want_pi else None
    v = torch.empty((B,), device=dev) if v is None else v
    L = _lib.lib()
    nbytes = int(L.az_heads_ws_bytes(B, K, A))
    ws = workspace(dev, max(nbytes, 64 << 20))
    _lib.check(L.az_heads_fwd(_p(hp), hp.stride(0), _p(hv), hv.stride(0), B, K, _p(wp), _p(bp), A,
                              _p(wv), _p(bv), _p(logp), _p(pi), _p(v), _p(ws),
                              ctypes.c_size_t(ws.numel()), _stream()), "az_heads_fwd")
    return logp, pi, v


class DeviceGraph:
    """A destination-sorted CSR graph resident in HBM, with the edge->dst map, the list of
    destinations that have in-edges, and the reverse (by-source) CSR the backward pass uses."""

    def __init__(self, rowptr, col, device="cuda"):
        import numpy as np
        rowptr = np.asarray(rowptr, np.int64)
        col = np.asarray(col, np.int64)
        V = len(rowptr) - 1
        deg = np.diff(rowptr)
        self.V, self.E = V, int(rowptr[-1])
        dst = np.repeat(np.arange(V), deg)
        rows = np.flatnonzero(deg > 0)
        self.D = len(rows)
        self.max_deg = int(deg.max()) if V else 0
        # max |src - dst| (the band kernel's condition: the row-major 32x32 grid gives 32)
        self.band = int(np.abs(col - np.repeat(np.arange(V), deg)).max()) if self.E else 0
        order = np.argsort(col, kind="stable")           # edges grouped by source
        src_rowptr = np.zeros(V + 1, np.int64)
        np.cumsum(np.bincount(col, minlength=V), out=src_rowptr[1:])
        dst_index = np.full(V, -1, np.int64)
        dst_index[rows] = np.arange(self.D)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.int32)).to(device)  # noqa: E731
        self.rowptr, self.col, self.edge_dst, self.dst_rows = t(rowptr), t(col), t(dst), t(rows)
        self.src_rowptr, self.src_edges, self.dst_index = t(src_rowptr), t(order), t(dst_index)
        self.c = Graph(V, self.E, self.rowptr.data_ptr(), self.col.data_ptr(),
                       self.edge_dst.data_ptr(), self.D, self.dst_rows.data_ptr(),
                       self.src_rowptr.data_ptr(), self.src_edges.data_ptr(),
                       self.dst_index.data_ptr(), self.max_deg, self.band)

    @staticmethod
    def star(n, device="cuda"):
        """The reference's implicit graph: row 0 <- rows 1..n-1 (gnn_utils.py:38-43)."""
        import numpy as np
        rowptr = np.full(n + 1, max(n - 1, 0), np.int64)
        rowptr[0] = 0
        return DeviceGraph(rowptr, np.arange(1, n), device)


def attn_score(g, P, H, b1, w2, b2, alpha=None):
    alpha = torch.empty((g.E,), device=P.device) if alpha is None else alpha
    L = _lib.lib()
    _lib.check(L.az_gnn_attn_score_fwd(ctypes.byref(g.c), _p(P), P.stride(0), H, _p(b1), _p(w2),
                                       _p(b2), _p(alpha), _stream()), "az_gnn_attn_score_fwd")
    return alpha


def aggregate(g, x, alpha, agg=None):
    F = x.shape[1]
    agg = torch.zeros_like(x) if agg is None else agg
    L = _lib.lib()
    _lib.check(L.az_gnn_aggregate_fwd(ctypes.byref(g.c), _p(x), x.stride(0), F, _p(alpha),
                                      _p(agg), agg.stride(0), _stream()), "az_gnn_aggregate_fwd")
    return agg


LAYER_KEYS = ("attention.0.weight", "attention.0.bias", "attention.2.weight", "attention.2.bias",
              "update_net.0.weight", "update_net.0.bias", "update_net.2.weight",
              "update_net.2.bias", "gate.0.weight", "gate.0.bias")


def layer_weights(Wl):
    """LayerW from a dict with GNNLayer state_dict suffixes."""
    return LayerW(*[Wl[k].data_ptr() for k in LAYER_KEYS])


def layer_grads(Gl):
    return LayerGrads(*[Gl[k].data_ptr() for k in LAYER_KEYS])


def layer_ws_bytes(g, F, H=128):
    return int(_lib.load().az_gnn_layer_ws_bytes(g.V, g.E, g.D, F, H))


def gnn_layer(g, x, Wl, out=None, ws=None, H=128, save=True):
    """One GNNLayer over graph g.  save=True (training): az_gnn_layer_fwd, which keeps the
    activations az_gnn_layer_bwd reads in `ws`; save=False (eval): az_gnn_layer_infer (the fused
    path on grid-shaped graphs).  Returns (x_out, ws)."""
    F = x.shape[1]
    out = torch.empty_like(x) if out is None else out
    L = _lib.lib()
    nbytes = layer_ws_bytes(g, F, H) if save else \
        int(L.az_gnn_layer_infer_ws_bytes(ctypes.byref(g.c), F, H))
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty((nbytes,), dtype=torch.uint8, device=x.device)
    lw = layer_weights(Wl)
    fn = L.az_gnn_layer_fwd if save else L.az_gnn_layer_infer
    _lib.check(fn(ctypes.byref(g.c), _p(x), F, H, ctypes.byref(lw), _p(out), _p(ws),
                  ctypes.c_size_t(ws.numel()), _stream()),
               "az_gnn_layer_fwd" if save else "az_gnn_layer_infer")
    return out, ws


def gnn_node_update(x, agg, Wl, dst_rows=None, out=None, save=None):
    """GNNLayer's gated node update alone (az_gnn_node_update_fwd, gnn_utils.py:18-28,67-74):
    out[d] = x[d] + sigmoid(Wg [x_d; agg_d] + bg) * (Wu2 relu(Wu1 [x_d; agg_d] + bu1) + bu2) on
    the destination rows dst_rows (int32 device tensor; None = every row), out = x elsewhere.
    Returns (out, save); save [3][D][F] feeds gnn_node_update_bwd."""
    V, F = x.shape
    D = V if dst_rows is None else int(dst_rows.numel())
    out = torch.empty_like(x) if out is None else out
    save = torch.empty((3, D, F), device=x.device) if save is None else save
    L = _lib.lib()
    ws = workspace(x.device, int(L.az_gnn_node_update_ws_bytes(D, F)))
    _lib.check(L.az_gnn_node_update_fwd(
        _p(x), _p(agg), V, F, D, None if dst_rows is None else _p(dst_rows),
        _p(Wl["gate.0.weight"]), _p(Wl["gate.0.bias"]), _p(Wl["update_net.0.weight"]),
        _p(Wl["update_net.0.bias"]), _p(Wl["update_net.2.weight"]), _p(Wl["update_net.2.bias"]),
        _p(out), _p(save), _p(ws), ctypes.c_size_t(ws.numel()), _stream()),
        "az_gnn_node_update_fwd")
    return out, save


NODE_UPDATE_KEYS = ("gate.0.weight", "gate.0.bias", "update_net.0.weight", "update_net.0.bias",
                    "update_net.2.weight", "update_net.2.bias")


def gnn_node_update_bwd(x, agg, Wl, save, dout, grads, dst_rows=None, dx=None, dagg=None):
    """az_gnn_node_update_bwd: dx (dout + the update's x-gradient on destination rows), dagg
    (destination rows; others zero here) and the six parameter gradients into grads (dict with
    NODE_UPDATE_KEYS).  Returns (dx, dagg)."""
    V, F = x.shape
    D = V if dst_rows is None else int(dst_rows.numel())
    dx = torch.empty_like(x) if dx is None else dx
    dagg = torch.zeros_like(x) if dagg is None else dagg
    L = _lib.lib()
    ws = workspace(x.device, int(L.az_gnn_node_update_bwd_ws_bytes(D, F)))
    _lib.check(L.az_gnn_node_update_bwd(
        _p(x), _p(agg), V, F, D, None if dst_rows is None else _p(dst_rows),
        _p(Wl["gate.0.weight"]), _p(Wl["update_net.0.weight"]), _p(Wl["update_net.2.weight"]),
        _p(save), _p(dout), _p(dx), _p(dagg), *[_p(grads[k]) for k in NODE_UPDATE_KEYS],
        _p(ws), ctypes.c_size_t(ws.numel()), _stream()), "az_gnn_node_update_bwd")
    return dx, dagg


def gnn_layer_ot(g, x, Wl, w0, b0, w2, b2, out=None, ws=None, H=128):
    """The network's last GNNLayer followed by output_transform, eval mode
    (az_gnn_layer_ot_infer: one band-kernel launch on band graphs).  Returns (y, ws)."""
    F = x.shape[1]
    out = torch.empty_like(x) if out is None else out
    L = _lib.lib()
    nbytes = int(L.az_gnn_layer_ot_infer_ws_bytes(ctypes.byref(g.c), F, H))
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty((nbytes,), dtype=torch.uint8, device=x.device)
    lw = layer_weights(Wl)
    _lib.check(L.az_gnn_layer_ot_infer(ctypes.byref(g.c), _p(x), F, H, ctypes.byref(lw),
                                       _p(w0), _p(b0), _p(w2), _p(b2), _p(out), _p(ws),
                                       ctypes.c_size_t(ws.numel()), _stream()),
               "az_gnn_layer_ot_infer")
    return out, ws


def gnn_source_proj(g, x, Wl, Ps=None, H=128):
    """Ps [V][H] = x W1[:, F:]^T (the fused layer path's first launch)."""
    Ps = torch.empty((g.V, H), device=x.device) if Ps is None else Ps
    L = _lib.lib()
    ws = workspace(x.device)
    _lib.check(L.az_gnn_source_proj_fwd(ctypes.byref(g.c), _p(x), x.shape[1], H,
                                        ctypes.byref(layer_weights(Wl)), _p(Ps), _p(ws),
                                        ctypes.c_size_t(ws.numel()), _stream()),
               "az_gnn_source_proj_fwd")
    return Ps


def gnn_layer_fused(g, x, Ps, Wl, out=None, H=128):
    """The fused layer kernel given Ps (the fused path's second launch)."""
    out = torch.empty_like(x) if out is None else out
    L = _lib.lib()
    _lib.check(L.az_gnn_layer_fused_fwd(ctypes.byref(g.c), _p(x), _p(Ps), x.shape[1], H,
                                        ctypes.byref(layer_weights(Wl)), _p(out), _stream()),
               "az_gnn_layer_fused_fwd")
    return out


def mlp2(x, w0, b0, w2, b2, hidden=None, out=None):
    M, F = x.shape
    hidden = torch.empty_like(x) if hidden is None else hidden
    out = torch.empty_like(x) if out is None else out
    L = _lib.lib()
    ws = workspace(x.device)
    _lib.check(L.az_mlp2_fwd(_p(x), M, F, _p(w0), _p(b0), _p(w2), _p(b2), _p(hidden), _p(out),
                             _p(ws), ctypes.c_size_t(ws.numel()), _stream()), "az_mlp2_fwd")
    return out, hidden


def transform_heads(x, w0, b0, w2, b2, wp, bp, wv, bv, hidden=None, y=None, logp=None, pi=None,
                    v=None, want_pi=True, want_y=True):
    """Per-row output_transform + heads (gnn_utils.py:115, Connect4GNN.py:48-57) in one C call:
    the second GEMM's split-K reduction is fused with the heads' first pass; with want_y=False
    y is never formed (the heads come from the GEMM's tiles, include/az_hip.h) and None returned.
    Returns (logp, pi, v, y, hidden)."""
    B, F = x.shape
    A = wp.shape[0]
    dev = x.device
    hidden = torch.empty_like(x) if hidden is None else hidden
    if want_y:
        y = torch.empty_like(x) if y is None else y
    else:
        y = None
    logp = torch.empty((B, A), device=dev) if logp is None else logp
    pi = (torch.empty((B, A), device=dev) if pi is None else pi) if want_pi else None
    v = torch.empty((B,), device=dev) if v is None else v
    L = _lib.lib()
    ws = workspace(dev, max(int(L.az_transform_heads_ws_bytes(B, F, A)), 96 << 20))
    _lib.check(L.az_transform_heads_fwd(_p(x), B, F, _p(w0), _p(b0), _p(w2), _p(b2), _p(wp),
                                        _p(bp), A, _p(wv), _p(bv), _p(hidden), _p(y), _p(logp),
                                        _p(pi), _p(v), _p(ws), ctypes.c_size_t(ws.numel()),
                                        _stream()), "az_transform_heads_fwd")
    return logp, pi, v, y, hidden


def c4_gnn_eval(boards, W, G, feat=None, hidden=None, y=None, logp=None, pi=None, v=None):
    """predict_with_gnn over a batch of 7x7 Connect4 boards (Connect4GNN.py:86-120 per row) as
    ONE az_c4_eval_fwd call: trunk -> output_transform -> heads.  The trunk also writes
    output_transform.0's A in the GEMM's split form and that GEMM's split-K reduce writes
    output_transform.2's, so neither GEMM launches a split of its own; bit-identical to
    c4_trunk + transform_heads.  W / G: the Connect4Net / PolicyValueGNN parameter dicts (their
    storage registered, e.g. FlatParams).  Returns (logp, pi, v)."""
    B = boards.shape[0]
    F = 3136
    A = W["fc_policy.weight"].shape[0]
    dev = boards.device
    assert boards.dtype == torch.int8 and boards.is_contiguous() and tuple(boards.shape[1:]) == (7, 7)
    for P_ in (W, G):
        if hasattr(P_, "sync"):
            P_.sync()       # FlatParams: announce torch-side weight writes (params.py)
    feat = torch.empty((B, F), device=dev) if feat is None else feat
    hidden = torch.empty((B, F), device=dev) if hidden is None else hidden
    y = torch.empty((B, F), device=dev) if y is None else y
    logp = torch.empty((B, A), device=dev) if logp is None else logp
    pi = torch.empty((B, A), device=dev) if pi is None else pi
    v = torch.empty((B,), device=dev) if v is None else v
    L = _lib.lib()
    ws = workspace(dev, max(int(L.az_transform_heads_ws_bytes(B, F, A)), 96 << 20))
    P = lambda t: t.data_ptr()  # noqa: E731
    desc = _lib.C4Eval(
        P(W["conv1.weight"]), P(W["conv1.bias"]), P(W["conv2.weight"]), P(W["conv2.bias"]),
        P(W["fc_policy.weight"]), P(W["fc_policy.bias"]), P(W["fc_value.weight"]),
        P(W["fc_value.bias"]), A, P(G["output_transform.0.weight"]),
        P(G["output_transform.0.bias"]), P(G["output_transform.2.weight"]),
        P(G["output_transform.2.bias"]), B, P(feat), P(hidden), P(y), P(logp), P(logp), P(ws),
        ws.numel())
    _lib.check(L.az_c4_eval_fwd(ctypes.byref(desc), _p(boards), B, None, None, _p(pi), _p(v),
                                _stream()), "az_c4_eval_fwd")
    return logp, pi, v


def linear_heads(x, w, b, wp, bp, wv, bv, y=None, logp=None, pi=None, v=None, want_pi=True,
                 want_y=True):
    """y = x w^T + b then the heads of y, with the GEMM's split-K reduction fused into the
    heads' first pass (the second half of transform_heads); want_y=False: y never formed
    (None returned).  Returns (logp, pi, v, y)."""
    B, F = x.shape
    A = wp.shape[0]
    dev = x.device
    if want_y:
        y = torch.empty_like(x) if y is None else y
    else:
        y = None
    logp = torch.empty((B, A), device=dev) if logp is None else logp
    pi = (torch.empty((B, A), device=dev) if pi is None else pi) if want_pi else None
    v = torch.empty((B,), device=dev) if v is None else v
    L = _lib.lib()
    ws = workspace(dev, max(int(L.az_transform_heads_ws_bytes(B, F, A)), 96 << 20))
    _lib.check(L.az_linear_heads_fwd(_p(x), B, F, _p(w), _p(b), _p(wp), _p(bp), A, _p(wv),
                                     _p(bv), _p(y), _p(logp), _p(pi), _p(v), _p(ws),
                                     ctypes.c_size_t(ws.numel()), _stream()),
               "az_linear_heads_fwd")
    return logp, pi, v, y


def adam(p, g, m, v, lr, step, beta1=0.9, beta2=0.999, eps=1e-8):
    L = _lib.lib()
    _lib.check(L.az_adam_step(_p(p), _p(g), _p(m), _p(v), p.numel(), lr, beta1, beta2, eps, step,
                             _stream()), "az_adam_step")


# ----------------------------------------------------------------------------- backward
def heads_loss_bwd(logp, v, target_pi, target_v, B_norm=None, loss_rows=None):
    B, A = logp.shape
    dl = torch.empty_like(logp)
    dv = torch.empty_like(v)
    L = _lib.lib()
    _lib.check(L.az_heads_loss_bwd(_p(logp), _p(v), _p(target_pi), _p(target_v), B, A,
                                   B_norm or B, _p(dl), _p(dv), _p(loss_rows), _stream()),
               "az_heads_loss_bwd")
    return dl, dv


def heads_bwd(dl, dv, hp, wp, wv, hv=None, grads=None, dh=None, dhv=None):
    """grads: dict with 'wp','bp','wv','bv' tensors to write (or None); dh: input-grad buffer
    (dhv None -> both heads summed into dh)."""
    hv = hp if hv is None else hv
    B, K = hp.shape
    A = wp.shape[0]
    L = _lib.lib()
    ws = workspace(hp.device)
    g = grads or {}
    dhv_t = dh if dhv is None else dhv
    _lib.check(L.az_heads_bwd(_p(dl), _p(dv), _p(hp), hp.stride(0), _p(hv), hv.stride(0), B, K,
                              _p(wp), A, _p(wv), _p(g.get("wp")), _p(g.get("bp")),
                              _p(g.get("wv")), _p(g.get("bv")), _p(dh),
                              dh.stride(0) if dh is not None else 0, _p(dhv_t),
                              dhv_t.stride(0) if dhv_t is not None else 0, _p(ws),
                              ctypes.c_size_t(ws.numel()), _stream()), "az_heads_bwd")


def colsum(X, out, beta=0.0):
    R, C = X.shape
    L = _lib.lib()
    ws = workspace(X.device)
    _lib.check(L.az_colsum(_p(X), R, C, X.stride(0), _p(out), beta, _p(ws),
                           ctypes.c_size_t(ws.numel()), _stream()), "az_colsum")
    return out


def dropout_mask(n, p, seed, device):
    m = torch.empty((n,), dtype=torch.uint8, device=device)
    L = _lib.lib()
    _lib.check(L.az_dropout_mask(_p(m), n, float(p), int(seed) & ((1 << 64) - 1), _stream()),
               "az_dropout_mask")
    return m


def mask_scale(x, mask, scale, out=None):
    out = torch.empty_like(x) if out is None else out
    L = _lib.lib()
    _lib.check(L.az_mask_scale(_p(x), _p(mask), float(scale), x.numel(), _p(out), _stream()),
               "az_mask_scale")
    return out


def nchw_drelu_to_pm(dy, y, B, C, HW, mask=None, scale=1.0, out=None):
    out = torch.empty((B * HW, C), device=dy.device) if out is None else out
    L = _lib.lib()
    _lib.check(L.az_nchw_drelu_to_pm(_p(dy), _p(y), _p(mask), float(scale), B, C, HW, _p(out),
                                     _stream()), "az_nchw_drelu_to_pm")
    return out


def im2col3x3(x, pad, ldc=None):
    is_i8 = x.dtype == torch.int8
    if is_i8:
        _need(x, torch.int8, "x")
        B, H, W = x.shape
        C = 1
    else:
        B, C, H, W = x.shape
    ldc = ldc or (C * 9 + 3) // 4 * 4
    Ho, Wo = H + 2 * pad - 2, W + 2 * pad - 2
    cols = torch.empty((B * Ho * Wo, ldc), device=x.device)
    L = _lib.lib()
    _lib.check(L.az_im2col3x3(_p(x), int(is_i8), B, C, H, W, pad, ldc, _p(cols), _stream()),
               "az_im2col3x3")
    return cols


def col2im3x3_drelu(dcols, a, pad):
    B, C, H, W = a.shape
    dz = torch.empty((B * H * W, C), device=a.device)
    L = _lib.lib()
    _lib.check(L.az_col2im3x3_drelu(_p(dcols), dcols.stride(0), _p(a), B, C, H, W, pad, _p(dz),
                                    _stream()), "az_col2im3x3_drelu")
    return dz


def gnn_layer_bwd(g, x, Wl, fwd_ws, dout, grads, dx=None, H=128):
    V, F = x.shape
    dx = torch.empty_like(x) if dx is None else dx
    L = _lib.lib()
    nbytes = int(L.az_gnn_layer_bwd_ws_bytes(g.V, g.E, g.D, F, H))
    ws = workspace(x.device, max(nbytes, 64 << 20))
    lw, lg = layer_weights(Wl), layer_grads(grads)
    _lib.check(L.az_gnn_layer_bwd(ctypes.byref(g.c), _p(x), F, H, ctypes.byref(lw), _p(fwd_ws),
                                  _p(dout), _p(dx), ctypes.byref(lg), _p(ws),
                                  ctypes.c_size_t(ws.numel()), _stream()), "az_gnn_layer_bwd")
    return dx


def mlp2_bwd(x, w0, w2, hidden, dy, grads, dx=None, want_dx=True):
    M, F = x.shape
    if want_dx and dx is None:
        dx = torch.empty_like(x)
    dh = torch.empty_like(x)
    L = _lib.lib()
    ws = workspace(x.device)
    _lib.check(L.az_mlp2_bwd(_p(x), M, F, _p(w0), _p(w2), _p(hidden), _p(dy),
                             _p(dx) if want_dx else None, _p(grads["w0"]), _p(grads["b0"]),
                             _p(grads["w2"]), _p(grads["b2"]), _p(dh), _p(ws),
                             ctypes.c_size_t(ws.numel()), _stream()), "az_mlp2_bwd")
    return dx

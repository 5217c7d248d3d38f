"""The reference's NeuralNet wrappers (Net.py:1-61 duck type) on libaz_hip.

Same constructor signature (game, args), same methods and return types as
connect4/Connect4Net.py:62-147, connect4/Connect4GNN.py:14-220, tictactoe/TicTacToeNet.py:50-104
and tictactoe/TicTacToeGNN.py:9-181, plus batched entry points (predict_batch,
predict_batch_with_gnn, predict_both) for lock-step self-play.  Checkpoints are the same
torch.save dict ({'state_dict': ..., 'gnn': ...}) with the same keys, so files move freely
between the reference and this implementation.
"""
import ctypes
import logging
import os

import numpy as np
import torch

from . import _lib, nets, ops, train as T
from .nets import boards_to_device

log = logging.getLogger(__name__)
# one-launch leaf hand-over timeouts in this process (each switches one evaluator to the
# four-launch path for good); bench.py reports it, so a degraded arena cannot go unnoticed
_LEAF_TIMEOUTS = [0]


def leaf_timeouts():
    """How many one-launch leaf evaluations timed out in this process (_Batch1Direct._call)."""
    return _LEAF_TIMEOUTS[0]


def _dev_array(rows, dtype, device):
    return torch.from_numpy(np.ascontiguousarray(np.array(rows), dtype=dtype)).to(device)


class PendingPrediction:
    """A batched prediction in flight on the device stream: boards went up from pinned host
    memory, the kernels are queued, the outputs come back into pinned host memory behind an
    event.  result() waits for that event only (the host keeps working meanwhile)."""

    def __init__(self, out_host, event, n, A, both):
        self.out_host, self.event, self.n, self.A, self.both = out_host, event, n, A, both

    def result(self):
        self.event.synchronize()
        out = self.out_host[:self.n].numpy().copy()
        A = self.A
        if self.both:
            return out[:, :A], out[:, A], out[:, A + 1:2 * A + 1], out[:, 2 * A + 1]
        return out[:, :A], out[:, A], None, None


class _PendingDirect:
    """A batched Connect4 prediction queued by _DirectBatch: the kernels write pi / v straight
    into mapped host memory; result() waits for the event and copies them out.

    The ring entry is owned through a token: only the prediction that took the entry may hand
    it back.  (A stale prediction object -- read long ago, dropped only when its variable is
    rebound -- must not free an entry a LATER prediction now holds: the next launch would then
    take the same host buffers and overwrite that prediction's outputs, which is what two
    self-play lanes did before the token.)  result() may be called more than once."""

    _tokens = iter(range(1, 1 << 62))

    def __init__(self, entry, views, event, n):
        # entry: the ring entry (its HostBuffer stays alive and reserved until result())
        self.entry, self.views, self.event, self.n = entry, views, event, n
        self.token = next(self._tokens)
        self.out = None
        entry["busy"] = True
        entry["owner"] = self.token

    def _release(self):
        if self.entry.get("owner") == self.token:
            self.entry["owner"] = None
            self.entry["busy"] = False

    def result(self):
        if self.out is None:
            self.event.synchronize()
            n = self.n
            self.out = tuple(None if a is None else a.numpy()[:n].copy() for a in self.views)
            self._release()
        return self.out

    def __del__(self):
        # dropped unread: the entry is free again once the device is done with it
        if self.entry.get("owner") == self.token:
            self.event.synchronize()
            self._release()


class _DirectBatch:
    """Batched predict_both / predict_batch for the 7x7 Connect4Net as ONE az_c4_eval_fwd call
    per batch (trunk + heads [+ output_transform + heads]): boards are read from and outputs
    written to mapped host memory (ops.HostBuffer, a ring of `depth` so that several batches can
    be in flight), device scratch is shared (the stream orders the batches).  Replaces ~10
    torch-level launches, a pinned H2D and a D2H copy per lock-step round."""

    def __init__(self, w, stream=None):
        self.w, self.cap, self.ring = w, 0, []
        self.stream = stream      # None: the current stream; else this stream (own scratch)
        self.fn = _lib.lib().az_c4_eval_fwd

    def _grow(self, n):
        w, dev, A, F = self.w, self.w.device, self.w.action_size, 3136
        cap = max(1024, 1 << (int(n) - 1).bit_length())
        torch.cuda.synchronize(dev)               # in-flight batches may use the old scratch
        self.feat = torch.empty((cap, F), device=dev)
        self.hidden = torch.empty((cap, F), device=dev)
        self.y = torch.empty((cap, F), device=dev)
        self.logp = torch.empty((cap, A), device=dev)
        self.glogp = torch.empty((cap, A), device=dev)
        L = _lib.lib()
        nb = max(int(L.az_transform_heads_ws_bytes(cap, F, A)), int(L.az_heads_ws_bytes(cap, F, A)))
        self.ws = torch.empty((nb,), dtype=torch.uint8, device=dev)
        W, G = w.nnet.params, w.gnn.params
        P = lambda t: t.data_ptr()  # noqa: E731
        self.desc = _lib.C4Eval(
            P(W["conv1.weight"]), P(W["conv1.bias"]), P(W["conv2.weight"]), P(W["conv2.bias"]),
            P(W["fc_policy.weight"]), P(W["fc_policy.bias"]), P(W["fc_value.weight"]),
            P(W["fc_value.bias"]), A, P(G["output_transform.0.weight"]),
            P(G["output_transform.0.bias"]), P(G["output_transform.2.weight"]),
            P(G["output_transform.2.bias"]), cap, P(self.feat), P(self.hidden), P(self.y),
            P(self.logp), P(self.glogp), P(self.ws), self.ws.numel())
        self.ring = []        # entries still held by unread predictions keep their buffers
        self.cap = cap

    def _entry(self):
        """A host staging set no unread prediction holds (a new one when all are held)."""
        for e in self.ring:
            if not e["busy"]:
                return e
        w, cap, A = self.w, self.cap, self.w.action_size
        off = [0, (cap * w.board_x * w.board_y + 255) // 256 * 256]
        for k in (A, 1, A, 1):
            off.append(off[-1] + (4 * cap * k + 255) // 256 * 256)
        hb = ops.HostBuffer(off[-1])
        e = {"busy": False, "hb": hb,
             "in": hb.view(0, torch.int8, (cap, w.board_x, w.board_y)),
             "out": [hb.view(off[1 + j], torch.float32, (cap, k) if k > 1 else (cap,))
                     for j, k in enumerate((A, 1, A, 1))]}
        self.ring.append(e)
        return e

    def launch(self, boards, both):
        boards = np.asarray(boards)
        n = boards.shape[0]
        if n > self.cap:
            self._grow(n)
        e = self._entry()
        hin, outs = e["in"], e["out"]
        hin.numpy()[:n] = boards
        pi, v, gpi, gv = outs if both else (outs[0], outs[1], None, None)
        s = self.stream if self.stream is not None else torch.cuda.current_stream(self.w.device)
        P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        rc = self.fn(ctypes.byref(self.desc), ctypes.c_void_p(hin.data_ptr()), n, P(pi), P(v),
                     P(gpi), P(gv), ctypes.c_void_p(s.cuda_stream))
        if rc:
            _lib.check(rc, "az_c4_eval_fwd")
        ev = torch.cuda.Event()
        ev.record(s)
        return _PendingDirect(e, (pi, v, gpi, gv), ev, n)


class _PinnedRing:
    """Pinned host staging buffers reused round-robin (`depth` predictions in flight)."""

    def __init__(self, depth=4):
        self.depth, self.i, self.bufs = depth, 0, {}

    def get(self, key, shape, dtype):
        k = (key, self.i % self.depth)
        b = self.bufs.get(k)
        if b is None or b.shape[0] < shape[0] or tuple(b.shape[1:]) != tuple(shape[1:]):
            b = torch.empty((max(shape[0], 1024),) + tuple(shape[1:]), dtype=dtype,
                            pin_memory=True)
            self.bufs[k] = b
        return b

    def advance(self):
        self.i += 1


class _Batch1Graph:
    """The whole batch-1 evaluation captured as ONE hipGraph: pinned host board -> H2D ->
    trunk -> heads [-> GNN tail] -> packed outputs -> D2H into pinned host memory.  MCTS asks
    for one leaf at a time wherever simulations depend on each other (the reference's
    MCTS.search, the arena's per-iteration trees), so this path is launch- and copy-latency
    bound; one replay replaces ~8 launches and two synchronous copies.  The kernels are the
    eager path's, so the outputs are bit-identical.  Parameters are updated in place (train,
    load_state_dict, restore), so the captured pointers stay valid.

    kind: "std" -> [pi, v], "gnn" -> [gnn_pi, gnn_v], "both" -> [pi, v, gnn_pi, gnn_v]."""

    def __init__(self, w, kind):
        dev = w.device
        A = w.action_size
        width = {"std": A + 1, "gnn": A + 1, "both": 2 * A + 2}[kind]
        # zero-copy staging (ops.HostBuffer): the trunk reads the board and the heads write
        # their pi / v straight from / into mapped host memory, so the graph has no copy
        # nodes; AZ_NO_ZEROCOPY=1 keeps the pinned-buffer + H2D / D2H copies instead
        self.host = None
        if os.environ.get("AZ_NO_ZEROCOPY", "0") in ("", "0"):
            try:
                self.host = ops.HostBuffer(256 + 4 * width)
            except RuntimeError:
                self.host = None
        if self.host is not None:
            self.h_in = self.host.view(0, torch.int8, (1, w.board_x, w.board_y))
            self.h_out = self.host.view(256, torch.float32, (1, width))
        else:
            self.h_in = torch.zeros((1, w.board_x, w.board_y), dtype=torch.int8, pin_memory=True)
            self.d_in = torch.zeros((1, w.board_x, w.board_y), dtype=torch.int8, device=dev)
            self.h_out = torch.zeros((1, width), dtype=torch.float32, pin_memory=True)
            self.d_out = torch.zeros((1, width), dtype=torch.float32, device=dev)
        zc = self.host is not None

        def body():
            if zc:
                o = self.h_out
                if kind in ("std", "both") and hasattr(w.nnet, "features_heads"):
                    f, _, _, _ = w.nnet.features_heads(self.h_in, pi=o[:, :A], v=o[:, A])
                elif kind in ("std", "both"):
                    f = w.nnet.features(self.h_in)
                    w.nnet.heads(f, pi=o[:, :A], v=o[:, A])
                else:
                    f = w.nnet.features(self.h_in)
                if kind in ("gnn", "both"):
                    c = 0 if kind == "gnn" else A + 1
                    nets.gnn_per_row_heads(w.nnet, w.gnn, f, pi=o[:, c:c + A], v=o[:, c + A])
                return
            self.d_in.copy_(self.h_in, non_blocking=True)
            f = w.nnet.features(self.d_in)
            parts = []
            if kind in ("std", "both"):
                _, pi, v = w.nnet.heads(f)
                parts += [pi, v[:, None]]
            if kind in ("gnn", "both"):
                _, gpi, gv = nets.gnn_per_row_heads(w.nnet, w.gnn, f)
                parts += [gpi, gv[:, None]]
            torch.cat(parts, dim=1, out=self.d_out)
            self.h_out.copy_(self.d_out, non_blocking=True)

        # the graph owns its workspace: the shared one is re-allocated when a large batch needs
        # more, which would leave a captured kernel pointing at freed memory
        self.ws = torch.empty((16 << 20,), dtype=torch.uint8, device=dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with ops.pinned_workspace(dev, self.ws):
            with torch.cuda.stream(side):
                body()                   # eager warm-up on the same buffers
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                body()
        self.dev = dev

    def run(self, board):
        self.h_in.numpy()[0] = board
        self.graph.replay()
        torch.cuda.current_stream(self.dev).synchronize()
        return self.h_out.numpy()[0].copy()


class _Batch1Direct:
    """Connect4 evaluation of up to `cap` boards as ONE C call (az_c4_eval_fwd: 1 + 3 direct
    launches) with zero-copy staging: the boards are read and pi / v written in place in mapped
    host memory.  Measured on MI355X, a hipGraph replay costs ~14 us of host time before its
    first kernel runs, more than these launches, which overlap the GPU work they queue.  Same
    kernels as the eager path (bit-identical outputs); parameters are read through the pointers
    fixed here, which stay valid because every update is in place.  kind as _Batch1Graph.

    Output layout in the host buffer: pi [cap][A], v [cap] (kind std/both), then gpi [cap][A],
    gv [cap] (kind gnn/both); with cap = 1 that is the packed [pi, v(, gpi, gv)] row run()
    returns.  cap = 8 serves the arena's speculative leaf batches (rows <= 8 take the same
    GEMV arithmetic as one row: mcts_native.ArenaPlayer, tests/test_gpu_selfplay.py)."""

    def __init__(self, w, kind, cap=1):
        dev = w.device
        A = w.action_size
        self.kind, self.A, self.cap = kind, A, cap
        std = kind in ("std", "both")
        gnn = kind in ("gnn", "both")
        width = (A + 1) * (int(std) + int(gnn))
        self.host = ops.HostBuffer(256 * cap + 4 * width * cap)
        self.h_in = self.host.view(0, torch.int8, (cap, w.board_x, w.board_y))
        self.h_out = self.host.view(256 * cap, torch.float32, (cap * width,))
        F = 3136
        self.feat = torch.empty((cap, F), device=dev)
        self.hidden = torch.empty((cap, F), device=dev) if gnn else None
        self.y = torch.empty((cap, F), device=dev) if gnn else None
        self.logp = torch.empty((cap, A), device=dev)
        self.glogp = torch.empty((cap, A), device=dev)
        self.ws = torch.empty((16 << 20,), dtype=torch.uint8, device=dev)
        W = w.nnet.params
        G = w.gnn.params if gnn else None
        P = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        self.desc = _lib.C4Eval(
            P(W["conv1.weight"]), P(W["conv1.bias"]), P(W["conv2.weight"]), P(W["conv2.bias"]),
            P(W["fc_policy.weight"]), P(W["fc_policy.bias"]), P(W["fc_value.weight"]),
            P(W["fc_value.bias"]), A,
            P(G["output_transform.0.weight"]) if gnn else None,
            P(G["output_transform.0.bias"]) if gnn else None,
            P(G["output_transform.2.weight"]) if gnn else None,
            P(G["output_transform.2.bias"]) if gnn else None,
            cap, P(self.feat), P(self.hidden), P(self.y), P(self.logp), P(self.glogp),
            P(self.ws), self.ws.numel())
        if kind == "both":
            # the one-launch form for 1-2 rows (c4_leaf_kernel): hand-over counters on the
            # device, zero between launches, and a host-visible timeout flag
            self.sync = torch.zeros(4096, dtype=torch.int32, device=dev)
            self.errbuf = ops.HostBuffer(256)
            self.err = self.errbuf.view(0, torch.int32, (1,))
            self.err.zero_()
            self.desc.sync = ctypes.c_void_p(self.sync.data_ptr())
            self.desc.err = ctypes.c_void_p(self.err.data_ptr())
            self.err_np = self.err.numpy()
        else:
            self.err_np = None
        L = _lib.lib()
        assert max(int(L.az_transform_heads_ws_bytes(cap, F, A)),
                   int(L.az_heads_ws_bytes(cap, F, A))) <= self.ws.numel()
        o = self.h_out.numpy()
        # views: pi [cap][A], v [cap], gpi [cap][A], gv [cap] (None where the kind has none)
        off, views = 0, []
        for on in (std, gnn):
            if on:
                views += [o[off:off + cap * A].reshape(cap, A), o[off + cap * A:off + cap * (A + 1)]]
                off += cap * (A + 1)
            else:
                views += [None, None]
        self.views = views
        self.args = (ctypes.byref(self.desc), ctypes.c_void_p(self.h_in.data_ptr()))
        self.outs = tuple(None if v is None else ctypes.c_void_p(v.ctypes.data) for v in views)
        self.fn = L.az_c4_eval_fwd
        self.dev = dev
        # the stream current at construction (the default stream, where train() updates the
        # parameters) serves every call: torch.cuda.current_stream() costs ~2.7 us per call
        self.stream = torch.cuda.current_stream(dev)
        self.sptr = ctypes.c_void_p(self.stream.cuda_stream)
        self.h_in_np = self.h_in.numpy()
        self.h_out_np = self.h_out.numpy()
        # keep the parameter tensors alive with the pointers taken above
        self._keep = (W, G)

    def _call(self, n):
        s = self.stream
        rc = self.fn(*self.args, n, *self.outs, self.sptr)
        if rc:
            _lib.check(rc, "az_c4_eval_fwd")
        s.synchronize()
        if self.err_np is not None and self.err_np[0]:
            # the one-launch form's hand-over timed out (its blocks were not all resident, e.g.
            # another process held CUs): discard the outputs, zero the counters, and evaluate
            # again with the four-launch path from now on
            self.sync.zero_()
            s.synchronize()
            self.err_np[0] = 0
            self.desc.sync = None
            self.desc.err = None
            self.err_np = None
            self.leaf_timeouts = getattr(self, "leaf_timeouts", 0) + 1
            _LEAF_TIMEOUTS[0] += 1
            log.warning("az_c4_eval_fwd: the one-launch leaf kernel's hand-over timed out (not "
                        "all its blocks were resident); this evaluator uses the four-launch path "
                        "from now on (%d timeout(s) in this process)", _LEAF_TIMEOUTS[0])
            rc = self.fn(*self.args, n, *self.outs, self.sptr)
            if rc:
                _lib.check(rc, "az_c4_eval_fwd")
            s.synchronize()

    def run(self, board):
        """One board -> the packed row [pi, v(, gpi, gv)] (cap 1)."""
        self.h_in_np[0] = board
        self._call(1)
        return self.h_out_np.copy()

    def run_rows(self, boards):
        """n <= cap boards -> (pi [n][A], v [n], gpi, gv) copies (None where the kind has none)."""
        n = len(boards)
        self.h_in_np[:n] = boards
        self._call(n)
        return tuple(None if v is None else v[:n].copy() for v in self.views)


def _direct_ok(w):
    """az_c4_eval_fwd covers the 7x7 Connect4Net (+ PolicyValueGNN output_transform)."""
    return (os.environ.get("AZ_B1_MODE", "direct") == "direct"
            and isinstance(w.nnet, nets.Connect4Net) and w.nnet.n == 7
            and os.environ.get("AZ_NO_ZEROCOPY", "0") in ("", "0"))


def _graphs_enabled():
    return os.environ.get("AZ_NO_GRAPH", "0") in ("", "0")


class NetWrapper:
    """Common body; subclasses choose the board network class and whether a GNN exists."""

    net_class = None
    has_gnn = False
    makedirs_on_save = True

    MAX_ACTIONS = 32      # the heads kernels keep a wave's A+1 weight chunks in registers

    def __init__(self, game, args):
        A = game.getActionSize()
        if A > self.MAX_ACTIONS:
            # rejected up front: MCTS would otherwise swallow every predict's error and play
            # a whole iteration on uniform priors before train() fails (MCTS.py:195-200)
            raise ValueError(f"{type(self).__name__}: action size {A} > {self.MAX_ACTIONS} is "
                             f"not supported by the HIP heads kernels (board {game.getBoardSize()})")
        self.device = nets.default_device()
        self.nnet = self.net_class(game, args, device=self.device)
        self.board_x, self.board_y = game.getBoardSize()
        self.action_size = game.getActionSize()
        self.args = args
        if self.has_gnn:
            self.feature_dim = self.nnet.feature_dim
            num_layers = nets._args_get(args, "gnn_layers", 2)
            self.gnn = nets.PolicyValueGNN(self.feature_dim, num_layers, device=self.device)
        self.train_seed = 0

    # -- evaluation ------------------------------------------------------------------------
    def _sync_params(self):
        """FlatParams.sync for both nets: the batch-1 and lock-step paths read the weights by
        pointer, so torch-side writes are announced here before they run."""
        self.nnet.params.sync()
        if self.has_gnn:
            self.gnn.params.sync()

    def _graph1(self, kind):
        """The batch-1 graph of `kind`, captured on first use (None when disabled)."""
        self._sync_params()
        if not _graphs_enabled():
            return None
        g = getattr(self, "_g1", None)
        if g is None:
            g = self._g1 = {}
        if kind not in g:
            self.nnet.eval()
            if self.has_gnn:
                self.gnn.eval()
            if _direct_ok(self):
                g[kind] = _Batch1Direct(self, kind, cap=8 if kind == "both" else 1)
            else:
                g[kind] = _Batch1Graph(self, kind)
        return g[kind]

    def _eval(self, boards, gnn):
        b = boards_to_device(boards, self.device)
        if b.dim() == 2:
            b = b.view(1, self.board_x, self.board_y)
        f = self.nnet.features(b)
        if gnn:
            _, pi, v = nets.gnn_per_row_heads(self.nnet, self.gnn, f)
            return pi, v
        _, pi, v = self.nnet.heads(f)
        return pi, v

    def predict(self, board, neighbor_states=None):
        """Net.predict: (pi float32[A], v float32) for one canonical board
        (Connect4GNN.py:59-84; `neighbor_states` is accepted and unused as in
        Connect4Net.py:110)."""
        self.nnet.eval()
        g = self._graph1("std")
        if g is not None:
            out = g.run(board)
            return out[:-1], out[-1]
        pi, v = self._eval(board, False)
        out = torch.cat([pi[0], v]).cpu().numpy()
        return out[:-1], out[-1]

    def predict_batch(self, boards):
        """Row-wise predict for [B,n,n] boards -> (pi float32[B,A], v float32[B])."""
        self.nnet.eval()
        if len(boards) == 1 and (g := self._graph1("std")) is not None:
            out = g.run(boards[0])
            return out[None, :-1], out[-1:]
        pi, v = self._eval(boards, False)
        return pi.cpu().numpy(), v.cpu().numpy()

    def _launch(self, boards, both, stream=None):
        """Queue a batched prediction; returns a PendingPrediction (see predict_*_async).
        stream: run it on that HIP stream with its own device scratch (the lock-step lanes give
        each lane a stream, so one lane's batch can overlap the other's on the GPU); the caller
        orders the stream after any parameter update (play_episodes_engine does)."""
        self._sync_params()
        if self.has_gnn and _direct_ok(self) and len(boards) > 0:
            directs = self.__dict__.setdefault("_directs", {})
            key = None if stream is None else stream.cuda_stream
            d = directs.get(key)
            if d is None:
                d = directs[key] = _DirectBatch(self, stream)
            self.nnet.eval()
            self.gnn.eval()
            return d.launch(boards, both)
        if not hasattr(self, "_ring"):
            self._ring = _PinnedRing()
        boards = np.asarray(boards)
        n = boards.shape[0]
        A = self.action_size
        hb = self._ring.get("in", (n,) + boards.shape[1:], torch.int8)
        hb[:n].numpy()[...] = boards
        b = hb[:n].to(self.device, non_blocking=True)
        self.nnet.eval()
        f = self.nnet.features(b)
        _, pi, v = self.nnet.heads(f)
        if both:
            self.gnn.eval()
            _, gpi, gv = nets.gnn_per_row_heads(self.nnet, self.gnn, f)
            out = torch.cat([pi, v[:, None], gpi, gv[:, None]], dim=1)
        else:
            out = torch.cat([pi, v[:, None]], dim=1)
        ho = self._ring.get("out", tuple(out.shape), torch.float32)
        ho[:n].copy_(out, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring.advance()
        return PendingPrediction(ho, ev, n, A, both)

    def predict_batch_async(self, boards):
        """predict_batch without waiting: .result() -> (pi, v, None, None)."""
        return self._launch(boards, False)

    def save_checkpoint(self, folder, filename):
        if self.makedirs_on_save and not os.path.exists(folder):
            os.makedirs(folder)
        filepath = os.path.join(folder, filename) if self.has_gnn else folder + "/" + filename
        payload = {"state_dict": self.nnet.params.cpu_state_dict()}
        if self.has_gnn:
            payload["gnn"] = self.gnn.params.cpu_state_dict()
        torch.save(payload, filepath)

    def load_checkpoint(self, folder, filename):
        filepath = os.path.join(folder, filename) if self.has_gnn else folder + "/" + filename
        checkpoint = torch.load(filepath, map_location="cpu", weights_only=True)
        self.nnet.load_state_dict(checkpoint["state_dict"])
        if self.has_gnn:
            if "gnn" in checkpoint:
                self.gnn.load_state_dict(checkpoint["gnn"])
            else:
                print(f"GNN state not found in {filepath}, initializing new GNN")

    # -- training --------------------------------------------------------------------------
    def _cnn_batch(self, examples):
        batch_idx = np.random.randint(0, len(examples), min(len(examples), self.args.batch_size))
        boards, pis, vs = list(zip(*[examples[i] for i in batch_idx]))
        return (_dev_array(boards, np.int8, self.device),
                _dev_array(pis, np.float32, self.device),
                _dev_array(np.array(vs).astype(np.float64), np.float32, self.device))

    def _gnn_batch(self, gnn_examples):
        batch_idx = np.random.randint(0, len(gnn_examples),
                                      min(len(gnn_examples), self.args.batch_size))
        batch = [gnn_examples[i] for i in batch_idx]
        boards = [b for b, _, _, _, _, _, _ in batch]
        pis = [p for _, _, _, _, p, _, _ in batch]
        vs = [v for _, _, _, _, _, v, _ in batch]
        return (_dev_array(boards, np.int8, self.device),
                _dev_array(pis, np.float32, self.device),
                _dev_array(np.array(vs).astype(np.float64), np.float32, self.device))

    def _train(self, examples, gnn_examples=None):
        """Connect4GNN.py:122-197: fresh Adam per call, `epochs` x (CNN step on a batch sampled
        with replacement by np.random.randint; GNN step on a second sample)."""
        lr = self.args.lr
        self._sync_params()
        if (nets._args_get(self.args, "train_parallel", "replicas") == "auto"
                and getattr(self, "_tp_auto", None) is None):
            from . import dist as D
            if D.world_rank()[0] > 1:
                self._tp_auto, self.train_parallel_probe = self._probe_train_parallel(
                    examples, gnn_examples)
        self.nnet.params.reset_adam()
        if self.has_gnn:
            self.gnn.params.reset_adam()
        for _ in range(self.args.epochs):
            self.nnet.train()
            if self.has_gnn:
                self.gnn.train()
            if examples:
                b, p, v = self._cnn_batch(examples)
                self.train_seed += 1
                if self._dp_world() > 1:
                    self._cnn_step_allreduce(b, p, v, lr)
                else:
                    T.cnn_step(self.nnet, b, p, v, lr, seed=self.train_seed)
            if self.has_gnn and gnn_examples and len(gnn_examples) > 0:
                b, p, v = self._gnn_batch(gnn_examples)
                self.train_seed += 1
                if self._dp_world() > 1:
                    T.gnn_step_dp(self.nnet, self.gnn, b, p, v, lr, seed=self.train_seed,
                                  grad_sync=nets._args_get(self.args, "gnn_grad_sync", "row0"))
                else:
                    T.gnn_step(self.nnet, self.gnn, b, p, v, lr, seed=self.train_seed)
        torch.cuda.current_stream().synchronize()


    def _dp_world(self):
        """>1 when the train steps are data-parallel over ranks (args.train_parallel ==
        "allreduce" under torch.distributed: CNN rows split + gradient all_reduce, the GNN step
        as train.gnn_step_dp); "replicas" (default) runs them whole everywhere; "auto" is
        whichever _probe_train_parallel measured faster on this process group."""
        from . import dist as D
        mode = nets._args_get(self.args, "train_parallel", "replicas")
        if mode == "auto":
            mode = getattr(self, "_tp_auto", None) or "replicas"
        if mode != "allreduce":
            return 1
        return D.world_rank()[0]

    def _probe_train_parallel(self, examples, gnn_examples):
        """train_parallel="auto" ('choose by measurement'): before the first
        train() under a process group of P > 1 ranks, time one gradient computation each way on
        this node -- the whole batch on every rank (replicas) against the data-parallel form
        with its collectives (the CNN rows sharded + the 188 KB all_reduce; the GNN step's
        sharded trunk, gathered features and the 78.7 MB output_transform all_reduce, or the
        478.6 MB one for gnn_grad_sync="flat") -- and keep the faster.  The Adam step is the same
        in both modes, so it is not timed.  The probe uses the first batch_size examples (no
        np.random draw: the training batches stay the reference's) and only writes gradient
        buffers, which every step overwrites.  Times are max over ranks, so every rank makes the
        same choice.  Returns (choice, {timings in ms})."""
        import time
        import torch.distributed as dist
        from . import dist as D
        world, rank = D.world_rank()
        sync = nets._args_get(self.args, "gnn_grad_sync", "row0")
        n = self.args.batch_size
        # every rank must probe the same jobs (each runs barriers and an all_reduce sized by
        # the job list): keep the kinds of examples every rank holds
        have = torch.tensor([1.0 if examples else 0.0,
                             1.0 if (self.has_gnn and gnn_examples) else 0.0],
                            dtype=torch.float64, device=self.device)
        dist.all_reduce(have, op=dist.ReduceOp.MIN)
        if have[0].item() == 0.0:
            examples = []
        if have[1].item() == 0.0:
            gnn_examples = []
        jobs = {}
        if examples:
            sel = examples[:n]
            b = _dev_array([e[0] for e in sel], np.int8, self.device)
            p = _dev_array([e[1] for e in sel], np.float32, self.device)
            v = _dev_array(np.array([e[2] for e in sel]).astype(np.float64), np.float32,
                           self.device)
            Bg = b.shape[0]
            r0, r1 = D.row_shard(Bg, world, rank)

            def cnn_dp():
                T.cnn_grads(self.nnet, b[r0:r1], p[r0:r1], v[r0:r1], seed=1, B_norm=Bg)
                D.allreduce_sum_(self.nnet.params.grad_flat)

            jobs["cnn"] = (lambda: T.cnn_grads(self.nnet, b, p, v, seed=1), cnn_dp)
        if self.has_gnn and gnn_examples:
            sel = gnn_examples[:n]
            gb = _dev_array([e[0] for e in sel], np.int8, self.device)
            gp = _dev_array([e[4] for e in sel], np.float32, self.device)
            gv = _dev_array(np.array([e[5] for e in sel]).astype(np.float64), np.float32,
                            self.device)
            jobs["gnn"] = (lambda: T.gnn_grads(self.nnet, self.gnn, gb, gp, gv, seed=1),
                           lambda: T.gnn_grads_dp(self.nnet, self.gnn, gb, gp, gv, seed=1,
                                                  grad_sync=sync))

        def timed(fn, reps=3):
            fn()                                      # first call: allocations, workspaces
            ts = []
            for _ in range(reps):
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts)) * 1e3

        names, vals = [], []
        for k, (rep, dp) in jobs.items():
            names += [f"{k}_replicas_ms", f"{k}_allreduce_ms"]
            vals += [timed(rep), timed(dp)]
        t = torch.tensor(vals, dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res = dict(zip(names, [round(float(x), 4) for x in t.tolist()]))
        rep_ms = sum(res[k] for k in names if k.endswith("_replicas_ms"))
        dp_ms = sum(res[k] for k in names if k.endswith("_allreduce_ms"))
        res.update(world=world, gnn_grad_sync=sync)
        return ("allreduce" if dp_ms < rep_ms else "replicas"), res

    def _cnn_step_allreduce(self, b, p, v, lr):
        """CNN step with the sampled rows split over ranks: each rank's loss is normalised by
        the GLOBAL batch, the flat gradient is summed with one all_reduce (RCCL), then every
        rank applies the identical Adam step.  The dropout mask is the global batch's mask
        (same counter-based seed), sliced to this rank's rows."""
        from . import dist as D
        world, rank = D.world_rank()
        Bg = b.shape[0]
        r0, r1 = D.row_shard(Bg, world, rank)
        F = self.nnet.feature_dim
        drop = float(getattr(self.nnet, "dropout", 0.0)) \
            if isinstance(self.nnet, nets.Connect4Net) else 0.0
        mask = None
        if drop > 0.0:
            mask = ops.dropout_mask(Bg * F, drop, self.train_seed, self.device)[r0 * F:r1 * F]
        P = self.nnet.params
        if r1 > r0:
            T.cnn_grads(self.nnet, b[r0:r1], p[r0:r1], v[r0:r1], seed=self.train_seed,
                        drop_mask=mask, B_norm=Bg)
        else:
            P.grad_flat.zero_()
        D.allreduce_sum_(P.grad_flat)
        T.adam_step(self.nnet, lr)

    def snapshot(self):
        """Device copy of every parameter buffer (Coach's temp checkpoint, in memory)."""
        snap = {"nnet": self.nnet.params.flat.clone()}
        if self.has_gnn:
            snap["gnn"] = self.gnn.params.flat.clone()
        return snap

    def restore(self, snap):
        self.nnet.params.copy_flat_(snap["nnet"])
        if self.has_gnn:
            self.gnn.params.copy_flat_(snap["gnn"])


class GNNWrapperMixin:
    """predict / predict_with_gnn pair of the GNN wrappers (Connect4GNN.py:59-120)."""

    has_gnn = True

    @property
    def batch_invariant_rows(self):
        """Largest batch whose predict_both rows are bit-identical to batch-1 calls: the 7x7
        Connect4 evaluator (az_c4_eval_fwd) computes every row of a batch of <= 8 with the
        batch-1 arithmetic (tests/test_gpu_selfplay.py); 0 = no such guarantee."""
        return 8 if _direct_ok(self) else 0

    def predict(self, board):
        return NetWrapper.predict(self, board)

    def predict_with_gnn(self, board):
        """GNN-enhanced prediction: a 1-row input, so the message-passing layers are the
        identity (gnn_utils.py:35-36) and only output_transform runs before the heads."""
        self.nnet.eval()
        self.gnn.eval()
        g = self._graph1("gnn")
        if g is not None:
            out = g.run(board)
            return out[:-1], out[-1]
        pi, v = self._eval(board, True)
        out = torch.cat([pi[0], v]).cpu().numpy()
        return out[:-1], out[-1]

    def predict_batch_with_gnn(self, boards):
        self.nnet.eval()
        self.gnn.eval()
        pi, v = self._eval(boards, True)
        return pi.cpu().numpy(), v.cpu().numpy()

    def predict_both(self, boards):
        """Standard and GNN predictions of a batch from ONE trunk pass (what MCTS.search asks
        for every new leaf, MCTS.py:169-174) -> (pi, v, gnn_pi, gnn_v), one host copy."""
        self.nnet.eval()
        self.gnn.eval()
        A = self.action_size
        g = self._graph1("both") if len(boards) <= 8 else None
        if isinstance(g, _Batch1Direct) and len(boards) > 0:
            return g.run_rows(np.asarray(boards))
        if len(boards) == 1 and g is not None:
            out = g.run(boards[0])[None]
            return out[:, :A], out[:, A], out[:, A + 1:2 * A + 1], out[:, 2 * A + 1]
        b = boards_to_device(boards, self.device)
        f = self.nnet.features(b)
        _, pi, v = self.nnet.heads(f)
        _, gpi, gv = nets.gnn_per_row_heads(self.nnet, self.gnn, f)
        out = torch.cat([pi, v[:, None], gpi, gv[:, None]], dim=1).cpu().numpy()
        return out[:, :A], out[:, A], out[:, A + 1:2 * A + 1], out[:, 2 * A + 1]

    def predict_both_async(self, boards, stream=None):
        """predict_both without waiting: .result() -> (pi, v, gnn_pi, gnn_v)."""
        return self._launch(boards, True, stream)

    def train(self, examples, gnn_examples=None):
        self._train(examples, gnn_examples)

    def extract_features(self, board_tensor):
        """Connect4GNN.py:31-46 / TicTacToeGNN.py:25-34 on device boards.  As in the reference,
        the Connect4 features go through dropout while `nnet.training` is set (the mask comes
        from the counter-based device RNG, not torch's generator)."""
        b = boards_to_device(board_tensor, self.device)
        if b.dim() == 2:
            b = b.view(1, self.board_x, self.board_y)
        f = self.nnet.features(b)
        p = float(getattr(self.nnet, "dropout", 0.0)) if isinstance(self.nnet, nets.Connect4Net) \
            else 0.0
        if self.nnet.training and p > 0.0:
            self.train_seed += 1
            mask = ops.dropout_mask(f.numel(), p, self.train_seed, f.device)
            f = ops.mask_scale(f, mask, 1.0 / (1.0 - p))
        return f

    def apply_policy_value_heads(self, features):
        """Connect4GNN.py:48-57 / TicTacToeGNN.py:36-45: features [B,F] on HBM ->
        (log_pi [B,A], v [B,1])."""
        logp, _, v = self.nnet.heads(features.contiguous(), want_pi=False)
        return logp, v.view(-1, 1)


class CNNWrapperMixin:
    has_gnn = False

    def train(self, examples):
        self._train(examples, None)

"""The lock-step parity checker (tests/lockstep_parity.py) on the host, no GPU: a network whose
rows depend on the batch they ride in (like the GPU's, whose GEMM split depends on M) drives
the native engine at several slot counts; every compared episode must replay exactly through
the reference loop, and the divergence classifier must pass rounding-sized differences and
FAIL a difference large enough to move a clear UCB decision."""
import hashlib

import numpy as np
import pytest

import lockstep_parity as LP
from test_mcts_golden import Args


class BatchNoiseNet:
    """Board-hash priors / values; rows of a batch of B > 1 are perturbed by `eps` times a
    hash of (board, B) -- batch-1 calls are not perturbed."""

    def __init__(self, A, eps):
        self.A, self.eps = A, eps

    def _row(self, board, kind, B):
        b = np.ascontiguousarray(board, np.int8).tobytes()
        h = hashlib.blake2b(b + bytes([kind]), digest_size=8).digest()
        r = np.random.default_rng(int.from_bytes(h, "little"))
        p = r.random(self.A) + 0.05
        v = r.random() * 2 - 1
        if B > 1 and self.eps:
            h2 = hashlib.blake2b(b + bytes([kind]) + B.to_bytes(4, "little"),
                                 digest_size=8).digest()
            q = np.random.default_rng(int.from_bytes(h2, "little"))
            p = p * (1 + self.eps * (q.random(self.A) - 0.5))
            v = float(np.clip(v + self.eps * (q.random() - 0.5), -1, 1))
        p = (p / p.sum()).astype(np.float32)
        return p, np.float32(v)

    def predict(self, board):
        return self._row(board, 0, 1)

    def predict_with_gnn(self, board):
        return self._row(board, 1, 1)

    def predict_both(self, boards):
        B = len(boards)
        s = [self._row(b, 0, B) for b in boards]
        g = [self._row(b, 1, B) for b in boards]
        return (np.stack([p for p, _ in s]), np.array([v for _, v in s], np.float32),
                np.stack([p for p, _ in g]), np.array([v for _, v in g], np.float32))


def _run(eps, G, n_eps=6, watch=4):
    from connect4.Connect4Game import Connect4Game
    game = Connect4Game(7)
    args = Args(numMCTSSims=15, cpuct=1.0, tempThreshold=15, use_gnn=True, expand_by=3)
    net = BatchNoiseNet(game.getActionSize(), eps)
    eps_list = list(range(n_eps))
    st = {}
    out, rows = LP.record_engine_rows(game, net, args, eps_list, {e: e for e in eps_list}, G,
                                      range(watch), threads=2, stats=st)
    reps = []
    for e in range(watch):
        seq = LP.sequential(game, net, args, e)
        reps.append(LP.compare_episode(game, args, e, seq, rows[e], out[e], tol=1e-5))
    return reps, st


def test_exact_rows_agree_everywhere():
    reps, st = _run(0.0, G=6)
    assert max(st["batch_rows"]) > 1
    for r in reps:
        assert r["replay_equals_engine"] and r["divergence"] is None, r


def test_rounding_sized_batch_noise_passes():
    """1e-7 relative noise per batch size: any divergence must be a near tie."""
    reps, _ = _run(1e-7, G=6)
    for r in reps:
        assert r["replay_equals_engine"], r
        assert r["divergence"] is None or r["divergence"]["near_tie"], r


def test_large_batch_noise_is_caught():
    """30 % noise per batch size moves clear decisions: the classifier must flag them."""
    reps, _ = _run(0.3, G=6)
    assert all(r["replay_equals_engine"] for r in reps)
    divs = [r["divergence"] for r in reps if r["divergence"] is not None]
    assert divs and any(not d["near_tie"] for d in divs), reps


def test_reference_trace_pinned_by_recorded_outputs():
    """G6c (mcts_c4_gnn_trace.npz, the reference's selection trace of episodes 0-15) against G6b
    (mcts_c4_gnn.npz: every network output the reference's episodes 0-2 requested): this repo's
    reference-shaped loop, fed G6b's recorded outputs, makes the same UCB selections -- state,
    action, Ns, and the score gap to 1e-6 -- as G6c recorded inside the reference's search, and
    the same examples, so the trace the GPU lock-step test compares against is the reference's
    search."""
    import json
    import os
    import lockstep_parity as LP
    from connect4.Connect4Game import Connect4Game
    from conftest import GOLDEN, golden
    from test_mcts_golden import Args, RecordedNet
    meta = json.load(open(os.path.join(GOLDEN, "mcts_c4_gnn.json")))
    trace = golden("mcts_c4_gnn_trace.npz")
    assert json.loads(str(trace["args"])) == meta["args"]
    net = RecordedNet(golden("mcts_c4_gnn.npz"), 7)
    game = Connect4Game(7)
    for ep in meta["episodes"]:
        e = ep["episode"]
        got = LP.sequential(game, net, Args(meta["args"]), e)
        ref = LP.reference_trace(trace, e)
        assert len(got["selects"]) == len(ref["selects"]), e
        for x, y in zip(got["selects"], ref["selects"]):
            assert (LP._state_key(x[0]), x[1], x[3]) == (y[0], y[1], y[3]), e
            # G6b stores the outputs as float32 (the GNN prior loses a few ulps of the
            # reference's value): the gaps agree to ~1e-8, far inside any near-tie bound
            assert x[2] == y[2] or abs(x[2] - y[2]) <= 1e-6, e
        assert LP.norm_std(got["std"]) == LP.norm_std(ref["std"]), e
        # init_v / exp_v / init_pi are network values and Q averages: G6b's float32 outputs
        # move them by ulps; board, player, visit-count targets and reward are exact
        assert LP._gnn_close(LP.norm_gnn(got["gnn"]), LP.norm_gnn(ref["gnn"]), 1e-6), e
        assert LP.first_divergence(ref, got, 1e-6, meta["args"]["cpuct"]) is None, e

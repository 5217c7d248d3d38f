"""Lock-step self-play vs the sequential reference loop, move by move (test infrastructure).

The north star asks for MCTS visit counts and action selection bit-exact with the reference on
a fixed seed (MCTS.py:151-240, Coach.py:27-79).  A lock-step game (selfplay.play_episodes_engine)
runs the same search as Coach.executeEpisode, but its leaf rows ride in batches of hundreds of
boards, and a row's bits depend on the batch (GEMM split / tile chosen by M): within 1e-5 of the
batch-1 call, not equal to it.  So a lock-step episode may leave the sequential episode -- and
the only legitimate way is a UCB near-tie that a 1e-5 network difference can flip.

This module proves that for every compared episode:

1. `record_engine_rows` plays the episodes in the native engine at G slots and keeps, per
   episode, every network row the engine consumed (board, pi, v, gnn_pi, gnn_v) in order.
2. `ReplayNet` serves exactly those rows to the reference-shaped Python loop
   (`sequential(...)`, Coach.executeEpisode after np.random.seed(e)): std rows in request order
   per board, the GNN row from the board's leaf evaluation.  The replay must reproduce the
   engine's examples EXACTLY (the engine == reference search, given the same outputs).
3. The replay and the sequential run with the batch-1 network both record every UCB selection
   (state, action, best-minus-second score gap, Ns).  `first_divergence` finds the first
   selection where they differ and checks the gap against `near_tie_bound`: the most a per-row
   output difference of `tol` can move a UCB score, u = Q + c P sqrt(N) / (1 + n) (Q an average
   of backed-up values: |dQ| <= tol; |dP| <= tol after renormalisation over valid moves, x2
   margin).  A divergence with a larger gap is a search bug, not rounding.
"""
import math
import zlib
from collections import defaultdict

import numpy as np


def near_tie_bound(tol, cpuct, ns):
    return 2.0 * (tol + 2.0 * tol * cpuct * math.sqrt(ns + 1))


def sequential(game, net, args, e):
    """Coach.executeEpisode after np.random.seed(e) (the reference loop) with `net`; records
    every UCB selection (state, action, gap between the best and second-best score, Ns)."""
    import Coach as C
    import MCTS as M
    coach = C.Coach.__new__(C.Coach)
    coach.game, coach.args, coach.nnet = game, args, net
    A = game.getActionSize()
    cpuct = args["cpuct"] if isinstance(args, dict) else args.cpuct
    selects = []
    orig_select = M.MCTS._select

    def rec_select(self, s):
        a = orig_select(self, s)
        us = []
        for b in range(A):
            if not self.Vs[s][b]:
                continue
            P = self.Ps[s][b]
            if (s, b) in self.Qsa:
                u = self.Qsa[(s, b)] + cpuct * P * math.sqrt(self.Ns[s]) / (1 + self.Nsa[(s, b)])
            else:
                u = cpuct * P * math.sqrt(self.Ns[s] + M.EPS)
            us.append(float(u))
        us.sort(reverse=True)
        selects.append((s, int(a), us[0] - us[1] if len(us) > 1 else math.inf, self.Ns[s]))
        return a

    M.MCTS._select = rec_select
    try:
        np.random.seed(e)
        coach.mcts = M.MCTS(game, net, args)
        std, gnn = coach.executeEpisode()
    finally:
        M.MCTS._select = orig_select
    return dict(selects=selects, std=std, gnn=gnn)


class _Caching:
    """Wraps a pending prediction so its result can be read twice (recorder + engine)."""

    def __init__(self, p):
        self.p, self.out = p, None
        if hasattr(p, "event"):
            self.event = p.event

    def result(self):
        if self.out is None:
            self.out = self.p.result()
        return self.out


def record_engine_rows(game, net, args, episodes, seeds, G, watch, threads=None, lanes=2,
                       stats=None):
    """play_episodes_engine with G slots; returns (results, rows) where rows[e] lists, for each
    watched episode e, the (board int8[n,n], pi, v, gpi, gv) rows the engine fed it, in order.
    Also reports the row counts per network call in stats['batch_rows']."""
    import selfplay as S
    watch = set(watch)
    rows = defaultdict(list)
    batch_rows = []
    orig_gather, orig_deliver = S._EpisodeLane.gather, S._EpisodeLane.deliver

    def gather(self):
        b = orig_gather(self)
        if b is not None:
            slots = self.eng.leaf_slots[:self.k]
            self._rec = (b.copy(), [self.running[int(s)] for s in slots])
            batch_rows.append(len(b))
        return b

    def deliver(self, pending):
        if pending is not None:
            pending = _Caching(pending)
            try:
                pi, v, gpi, gv = pending.result()
            except Exception:
                pass
            else:
                boards, eps = self._rec
                for i, e in enumerate(eps):
                    if e in watch:
                        rows[e].append((boards[i].copy(), np.array(pi[i]), np.float32(v[i]),
                                        np.array(gpi[i]) if gpi is not None else None,
                                        np.float32(gv[i]) if gv is not None else None))
        return orig_deliver(self, pending)

    S._EpisodeLane.gather, S._EpisodeLane.deliver = gather, deliver
    try:
        out = S.play_episodes_engine(game, net, args, episodes, seeds, parallel_games=G,
                                     threads=threads, lanes=lanes, stats=stats)
    finally:
        S._EpisodeLane.gather, S._EpisodeLane.deliver = orig_gather, orig_deliver
    if stats is not None:
        stats["batch_rows"] = batch_rows
    return out, rows


class ReplayNet:
    """Serves one episode's recorded engine rows to the batch-1 reference plumbing: predict(b)
    returns b's std rows in the order the engine consumed them, predict_with_gnn(b) the GNN row
    of b's leaf evaluation (a board is a new leaf at most once per episode tree)."""

    def __init__(self, rows):
        self.std = defaultdict(list)
        self.gnn = {}
        for b, pi, v, gpi, gv in rows:
            k = np.asarray(b, np.int8).tobytes()
            self.std[k].append((pi, v))
            if gpi is not None and k not in self.gnn:
                self.gnn[k] = (gpi, gv)
        self.used = defaultdict(int)

    def predict(self, board):
        k = np.asarray(board, np.int8).tobytes()
        i = self.used[k]
        self.used[k] += 1
        lst = self.std[k]
        p, v = lst[min(i, len(lst) - 1)]
        return np.array(p, np.float32), np.float32(v)

    def predict_with_gnn(self, board):
        p, v = self.gnn[np.asarray(board, np.int8).tobytes()]
        return np.array(p, np.float32), np.float32(v)


def norm_std(std):
    return [(np.asarray(b).astype(int).tolist(), [float(x) for x in p], float(z))
            for b, p, z in std]


def norm_gnn(gnn):
    return [(np.asarray(x[0]).astype(int).tolist(), int(x[1]), [float(t) for t in x[2]],
             float(x[3]), [float(t) for t in x[4]], float(x[5]), float(x[6])) for x in gnn]


def _gnn_close(x, y, tol):
    """GNN examples (MCTS.expand_tree targets, MCTS.py:120-146): board, player, exp_pi (visit
    counts) and reward exact; init_pi, init_v and exp_v are network outputs / Q averages, equal
    within the network tolerance."""
    if len(x) != len(y):
        return False
    for a, b in zip(x, y):
        if (a[0], a[1], a[4], a[6]) != (b[0], b[1], b[4], b[6]):
            return False
        if max(abs(u - w) for u, w in zip(a[2], b[2])) > tol or abs(a[3] - b[3]) > tol or \
                abs(a[5] - b[5]) > tol:
            return False
    return True


def _state_key(s):
    """A selection's state as the reference trace stores it (tests/golden/make_goldens.py g6c:
    crc32 of the state bytes), so live runs (bytes) compare with the recorded trace (ints)."""
    return zlib.crc32(s) if isinstance(s, (bytes, bytearray)) else int(s)


def reference_trace(z, e):
    """Episode e of the reference's recorded search (G6c, mcts_c4_gnn_trace.npz) in the form
    `sequential` returns: selects (state crc32, action, gap, Ns), std and GNN examples."""
    i = int(np.flatnonzero(z["episodes"] == e)[0])
    a, b = int(z["sel_off"][i]), int(z["sel_off"][i + 1])
    selects = list(zip(z["sel_state_crc32"][a:b].tolist(), z["sel_action"][a:b].tolist(),
                       z["sel_gap"][a:b].tolist(), z["sel_ns"][a:b].tolist()))
    a, b = int(z["std_off"][i]), int(z["std_off"][i + 1])
    std = [(z["std_board"][j], z["std_pi"][j], float(z["std_z"][j])) for j in range(a, b)]
    a, b = int(z["gnn_off"][i]), int(z["gnn_off"][i + 1])
    gnn = [(z["gnn_board"][j], int(z["gnn_player"][j]), z["gnn_init_pi"][j],
            np.float32(z["gnn_init_v"][j]), z["gnn_exp_pi"][j], float(z["gnn_exp_v"][j]),
            float(z["gnn_reward"][j])) for j in range(a, b)]
    return dict(selects=selects, std=std, gnn=gnn)


def first_divergence(seq, rep, tol, cpuct):
    """Compare two recorded runs of one episode.  Returns None when they agree (identical UCB
    selections, identical std examples, GNN examples equal up to `tol` in their network-valued
    fields), else a dict with the first differing selection, its gaps in both runs, the bound
    and `near_tie` (gap of the sequential run <= bound)."""
    same_std = norm_std(seq["std"]) == norm_std(rep["std"])
    same_gnn = _gnn_close(norm_gnn(seq["gnn"]), norm_gnn(rep["gnn"]), tol)
    k = next((j for j, (x, y) in enumerate(zip(seq["selects"], rep["selects"]))
              if (_state_key(x[0]), x[1]) != (_state_key(y[0]), y[1])), None)
    # examples carry the game's final reward: compare (board, pi) to find the first move apart
    a = [x[:2] for x in norm_std(seq["std"])]
    b = [x[:2] for x in norm_std(rep["std"])]
    n = min(len(a), len(b))
    first_ex = next((i for i in range(n) if a[i] != b[i]), n)
    if k is None and len(seq["selects"]) == len(rep["selects"]):
        if same_std and same_gnn:
            return None
        # same selections, different examples: a value / target moved by more than tol
        return {"select_index": None, "first_example": first_ex, "near_tie": False,
                "why": "examples differ beyond tol with identical selections"}
    if k is None:
        return {"select_index": None, "first_example": first_ex, "near_tie": False,
                "why": "one run made more selections with identical prefixes"}
    s, _, gap_seq, ns = seq["selects"][k]
    gap_rep = rep["selects"][k][2]
    bound = near_tie_bound(tol, cpuct, ns)
    return {"select_index": k, "first_example": first_ex, "first_move": first_ex // 2,
            "gap_sequential": gap_seq, "gap_lockstep": gap_rep, "ns": int(ns), "bound": bound,
            "near_tie": bool(gap_seq <= bound)}


def compare_episode(game, args, e, seq, rows, engine_result, tol):
    """Replays episode e's engine rows through the reference loop (must equal the engine's
    examples), then locates and classifies the first divergence from the sequential run."""
    rep = sequential(game, ReplayNet(rows), args, e)
    replay_exact = (norm_std(rep["std"]) == norm_std(engine_result[0]) and
                    norm_gnn(rep["gnn"]) == norm_gnn(engine_result[1]))
    cpuct = args["cpuct"] if isinstance(args, dict) else args.cpuct
    div = first_divergence(seq, rep, tol, cpuct)
    moves = len(seq["std"]) // 2
    agree = moves if div is None else min(moves, div["first_example"] // 2)
    return {"episode": e, "replay_equals_engine": replay_exact, "moves": moves,
            "agreeing_moves": agree, "divergence": div}

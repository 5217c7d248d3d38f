"""Native MCTS (libaz_mcts.so, include/az_mcts.h) behind the reference's MCTS interface.

`Engine` binds the C-ABI with ctypes.  `NativeMCTS` is one game slot of an engine, with the
generator methods `getActionProb_g` / `expand_tree_g` that Coach.episode_g drives, so the
episode logic (temperature, sampling, symmetries, GNN targets) is the same Python code as the
sequential path, while the searches (MCTS.py:151-240) and the rules they call run natively
for every slot at once.  The generators yield

    ("search", board_int8, sims)   run `sims` searches from this root (engine-side)
    ("predict", board_int64)       the root's standard prediction (MCTS.py:108-113)

and selfplay.play_episodes_native serves both kinds for all slots with one batched network
call per round.  Q values come back with their Python type (int / float / np.float32), so the
root statistics and everything computed from them are the reference's bit for bit
(tests/test_native_mcts.py).
"""
import ctypes
import os

import numpy as np

import nn_fallback

EPS = 1e-8
HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "azhip", "libaz_mcts.so")
# AZ_AB_MCTS_LIB=<file in azhip/>: an A/B build of the engine at another revision (tools/)
if os.environ.get("AZ_AB_MCTS_LIB"):
    LIB_PATH = os.path.join(HERE, "azhip", os.path.basename(os.environ["AZ_AB_MCTS_LIB"]))

GAME_CONNECT4, GAME_TICTACTOE = 0, 1
TAG_NONE, TAG_INT, TAG_FLOAT, TAG_F32 = -1, 0, 1, 2

_lib = None

_P = ctypes.c_void_p
_SIGS = {
    "az_mcts_last_error": (ctypes.c_char_p, []),
    "az_mcts_create": (_P, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                            ctypes.c_int]),
    "az_mcts_destroy": (None, [_P]),
    "az_mcts_action_size": (ctypes.c_int, [_P]),
    "az_mcts_reset": (ctypes.c_int, [_P, ctypes.c_int]),
    "az_mcts_clear_predictions": (ctypes.c_int, [_P, ctypes.c_int]),
    "az_mcts_begin": (ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.c_int]),
    "az_mcts_remaining": (ctypes.c_int, [_P, ctypes.c_int]),
    "az_mcts_abandon": (ctypes.c_int, [_P, ctypes.c_int]),
    "az_mcts_remaining_all": (ctypes.c_int, [_P, _P]),
    "az_mcts_collect": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, ctypes.c_int]),
    "az_mcts_feed": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, ctypes.c_int]),
    "az_mcts_feed_collect": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, _P, _P,
                                            ctypes.c_int, ctypes.c_int]),
    "az_mcts_cache_put": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, _P]),
    "az_mcts_cache_clear": (ctypes.c_int, [_P]),
    "az_mcts_collect_spec": (ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.c_int]),
    "az_mcts_feed_spec": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, ctypes.c_int]),
    "az_mcts_cache_stats": (ctypes.c_int, [_P, _P]),
    "az_mcts_root_edges": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P]),
    "az_mcts_get_std": (ctypes.c_int, [_P, ctypes.c_int, _P, _P]),
    "az_mcts_set_std": (ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.c_float]),
    "az_mcts_tree_stats": (ctypes.c_int, [_P, ctypes.c_int, _P]),
    "az_game_ended": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P, _P, _P]),
    "az_game_valids": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P, _P]),
    "az_game_next_canonical": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P, ctypes.c_int, _P]),
    "az_game_children": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P, ctypes.c_int, _P]),
    "az_np_pairwise_sum": (ctypes.c_double, [_P, ctypes.c_int]),
    "az_mcts_episode_begin": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int]),
    "az_mcts_episode_finished": (ctypes.c_int, [_P, _P, ctypes.c_int]),
    "az_mcts_episode_moves": (ctypes.c_int, [_P, ctypes.c_int]),
    "az_mcts_episode_record": (ctypes.c_int, [_P, ctypes.c_int] + [_P] * 13),
    "az_mcts_episode_targets": (ctypes.c_int, [_P, ctypes.c_int] + [_P] * 4),
    "az_mcts_episodes_moves": (ctypes.c_int, [_P, _P, ctypes.c_int, _P]),
    "az_mcts_episode_records": (ctypes.c_int, [_P, _P, ctypes.c_int] + [_P] * 17),
    "az_rng_test": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, _P, ctypes.c_int,
                                   _P]),
    "az_rng_doubles": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_int, _P]),
}


def lib():
    """The engine library (built by __graft_entry__.build() / azhip.build.build_host())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `python -m azhip.build` (or "
                               "__graft_entry__.build()) first")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def _ptr(a):
    # a plain int is accepted for a c_void_p argument (cheaper than a.ctypes.data)
    return a.__array_interface__["data"][0]


def _check(rc, what):
    if rc < 0:
        raise RuntimeError(f"{what}: {lib().az_mcts_last_error().decode()}")
    return rc


def game_kind(game):
    """(engine game id, n) for the two registered games; ValueError for anything else."""
    name = type(game).__name__
    if name == "Connect4Game":
        return GAME_CONNECT4, int(game.board_size)
    if name == "TicTacToeGame":
        return GAME_TICTACTOE, int(game.n)
    raise ValueError(f"native MCTS supports Connect4Game / TicTacToeGame, not {name}")


def typed_q(tag, x):
    """The Python object the reference's Qsa holds."""
    if tag == TAG_INT:
        return int(x)
    if tag == TAG_FLOAT:
        return float(x)
    return np.float32(x)


class Engine:
    """One libaz_mcts engine: `slots` concurrent game trees of one game kind."""

    def __init__(self, game, slots, cpuct, use_gnn):
        self.kind, self.n = game_kind(game)
        self.cells = self.n * self.n
        self.slots = slots
        self.use_gnn = bool(use_gnn)
        h = lib().az_mcts_create(self.kind, self.n, slots, float(cpuct), int(self.use_gnn))
        if not h:
            raise RuntimeError("az_mcts_create: " + lib().az_mcts_last_error().decode())
        self.h = ctypes.c_void_p(h)
        self.A = lib().az_mcts_action_size(self.h)
        self.leaf_boards = np.zeros((slots, self.n, self.n), np.int8)
        self.leaf_slots = np.zeros(slots, np.int32)
        self._rem = np.zeros(slots, np.int32)
        self._nsa = np.zeros(self.A, np.int32)
        self._q = np.zeros(self.A, np.float64)
        self._tag = np.zeros(self.A, np.int8)
        self._b = np.zeros((self.n, self.n), np.int8)
        self._pb, self._ps, self._pr = (_ptr(self.leaf_boards), _ptr(self.leaf_slots),
                                        _ptr(self._rem))
        self._pn, self._pq, self._pt, self._pbb = (_ptr(self._nsa), _ptr(self._q),
                                                   _ptr(self._tag), _ptr(self._b))
        # small feeds / cache puts (the arena's batch-1 leaves) go through persistent staging
        # buffers with pointers taken once: a numpy pointer lookup costs ~1.5 us, more than the
        # copy of a few rows
        self._scap = 64
        self._stage = [np.zeros((self._scap, self.A), np.float32), np.zeros(self._scap, np.float32),
                       np.zeros((self._scap, self.A), np.float32), np.zeros(self._scap, np.float32)]
        self._sptr = [_ptr(a) for a in self._stage]
        self._sboards = np.zeros((self._scap, self.n, self.n), np.int8)
        self._psb = _ptr(self._sboards)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _lib is not None:
            _lib.az_mcts_destroy(h)
            self.h = None

    @staticmethod
    def _b8(board):
        return np.ascontiguousarray(board, dtype=np.int8)

    def _bp(self, board):
        """Pointer to an int8 copy of `board` in a reused buffer."""
        self._b[...] = board
        return self._pbb

    def reset(self, slot):
        _check(lib().az_mcts_reset(self.h, slot), "az_mcts_reset")

    def clear_predictions(self, slot):
        _check(lib().az_mcts_clear_predictions(self.h, slot), "az_mcts_clear_predictions")

    def begin(self, slot, board, sims):
        b = self._b8(board)
        _check(lib().az_mcts_begin(self.h, slot, _ptr(b), int(sims)), "az_mcts_begin")

    def remaining(self, slot):
        return _check(lib().az_mcts_remaining(self.h, slot), "az_mcts_remaining")

    def abandon(self, slot):
        _check(lib().az_mcts_abandon(self.h, slot), "az_mcts_abandon")

    def remaining_all(self):
        """int32 [slots] view (overwritten by the next call)."""
        _check(lib().az_mcts_remaining_all(self.h, self._pr), "az_mcts_remaining_all")
        return self._rem

    def collect(self, threads=1):
        """-> number of leaves; boards in self.leaf_boards[:k], slots in self.leaf_slots[:k]."""
        return _check(lib().az_mcts_collect(self.h, self._pb, self._ps, self.slots,
                                            int(threads)), "az_mcts_collect")

    def feed(self, k, pi=None, v=None, gpi=None, gv=None, failed=False):
        """Network outputs for the last collect's k leaves (or failed=True: the reference's
        uniform-priors / v=0 path).  Returns the number of episode-mode slots whose expand_tree
        root prediction was among the failed requests: those episodes are aborted (the
        reference's root predict is unguarded, MCTS.py:108-113) and the caller must raise."""
        k = int(k)
        if failed:
            return _check(lib().az_mcts_feed(self.h, k, None, None, None, None, 1), "az_mcts_feed")
        ptrs = self._rows_ptrs("Engine.feed", k, pi, v, gpi, gv, at_least=True)
        return _check(lib().az_mcts_feed(self.h, k, *ptrs, 0), "az_mcts_feed")

    def feed_collect(self, k, pi, v, gpi=None, gv=None, threads=1):
        """feed(k, pi, v, gpi, gv) then collect(threads) in one native pass (az_mcts_feed_collect);
        -> the new leaf count, boards in self.leaf_boards[:n]."""
        ptrs = self._rows_ptrs("Engine.feed_collect", int(k), pi, v, gpi, gv, at_least=True)
        return _check(lib().az_mcts_feed_collect(self.h, int(k), *ptrs, self._pb, self._ps,
                                                 self.slots, int(threads)),
                      "az_mcts_feed_collect")

    def _rows_ptrs(self, what, k, pi, v, gpi, gv, at_least):
        """Checked float32 row pointers for pi / v (/ gpi / gv when use_gnn): the C side reads
        pi + i*A for i < k, so shapes are verified before any pointer escapes.  Up to 64 rows
        are copied into the staging buffers (fixed pointers), larger batches are passed as
        contiguous float32 arrays (kept alive in self._keep until the next call)."""
        arrs = (pi, v, gpi, gv) if self.use_gnn else (pi, v)
        out = [None, None, None, None]
        self._keep = []
        for j, (name, a) in enumerate(zip(("pi", "v", "gpi", "gv"), arrs)):
            if a is None:
                raise ValueError(f"{what}: {name} missing")
            nd = 2 if j % 2 == 0 else 1
            sh = np.shape(a)
            if len(sh) != nd or (sh[0] < k if at_least else sh[0] != k) or \
                    (nd == 2 and sh[1] != self.A):
                raise ValueError(f"{what}: {name} has shape {sh}, need "
                                 f"({'>=' if at_least else ''}{k}{', %d' % self.A if nd == 2 else ''})")
            if k <= self._scap:
                self._stage[j][:k] = a[:k]
                out[j] = self._sptr[j]
            else:
                c = np.ascontiguousarray(a[:k], dtype=np.float32)
                self._keep.append(c)
                out[j] = _ptr(c)
        return out

    def cache_put(self, boards, pi, v, gpi=None, gv=None):
        """Rows for boards the search has not reached yet (see az_mcts_cache_put): a later new
        leaf on one of them is expanded inside collect().  Rows must be bit-identical to the
        board's own evaluation."""
        k = len(boards)
        if k == 0:
            return
        ptrs = self._rows_ptrs("Engine.cache_put", k, pi, v, gpi, gv, at_least=False)
        if k <= self._scap:
            self._sboards[:k] = boards
            pb = self._psb
        else:
            b = np.ascontiguousarray(boards, dtype=np.int8)
            self._keep.append(b)
            pb = _ptr(b)
        _check(lib().az_mcts_cache_put(self.h, k, pb, *ptrs), "az_mcts_cache_put")

    def collect_spec(self, slot, boards_ptr, cap):
        """Next new leaf of `slot` + up to cap - 1 speculative children into the int8 buffer at
        boards_ptr (see az_mcts_collect_spec) -> row count, 0 when the searches are done."""
        return _check(lib().az_mcts_collect_spec(self.h, slot, boards_ptr, int(cap)),
                      "az_mcts_collect_spec")

    def feed_spec(self, k, pi=None, v=None, gpi=None, gv=None, failed=False):
        """Rows for the last collect_spec's k boards (row 0 = the leaf)."""
        if failed:
            return _check(lib().az_mcts_feed_spec(self.h, k, None, None, None, None, 1),
                          "az_mcts_feed_spec")
        ptrs = self._rows_ptrs("Engine.feed_spec", k, pi, v, gpi, gv, at_least=False)
        return _check(lib().az_mcts_feed_spec(self.h, k, *ptrs, 0), "az_mcts_feed_spec")

    def cache_stats(self):
        """-> (rows held, leaves expanded from them)."""
        out = np.zeros(2, np.int64)
        _check(lib().az_mcts_cache_stats(self.h, _ptr(out)), "az_mcts_cache_stats")
        return int(out[0]), int(out[1])

    def root_edges(self, slot, board):
        """-> (nsa list[int], q list[float64], tags list[int])."""
        _check(lib().az_mcts_root_edges(self.h, slot, self._bp(board), self._pn, self._pq,
                                        self._pt), "az_mcts_root_edges")
        return self._nsa.tolist(), self._q.tolist(), self._tag.tolist()

    def get_std(self, slot, board):
        b = self._b8(board)
        v = np.zeros(1, np.float32)
        r = _check(lib().az_mcts_get_std(self.h, slot, _ptr(b), _ptr(v)), "az_mcts_get_std")
        return v[0] if r == 1 else None

    def set_std(self, slot, board, v):
        b = self._b8(board)
        _check(lib().az_mcts_set_std(self.h, slot, _ptr(b), float(v)), "az_mcts_set_std")

    # -- episode mode ----------------------------------------------------------------------
    def episode_begin(self, slot, seed, sims, expand_by, temp_threshold):
        _check(lib().az_mcts_episode_begin(self.h, slot, int(seed) & 0xFFFFFFFF, int(sims),
                                           int(expand_by), int(temp_threshold)),
               "az_mcts_episode_begin")

    def episodes_finished(self):
        if not hasattr(self, "_fin"):
            self._fin = np.zeros(self.slots, np.int32)
            self._pfin = _ptr(self._fin)
        k = _check(lib().az_mcts_episode_finished(self.h, self._pfin, self.slots),
                   "az_mcts_episode_finished")
        return self._fin[:k].tolist()

    _REC = (("boards", np.int8, "C"), ("cur", np.int8, 1), ("temp", np.int8, 1),
            ("action", np.int32, 1), ("pi", np.float64, "A"), ("init_nsa", np.int32, "A"),
            ("init_has", np.int8, "A"), ("std_v", np.float32, 1), ("exp_nsa", np.int32, "A"),
            ("exp_q", np.float64, "A"), ("exp_tag", np.int8, "A"))
    _TGT = (("init_policy", np.float64, "A"), ("exp_policy", np.float64, "A"),
            ("exp_value_tag", np.int8, 1), ("exp_value", np.float64, 1))

    def episode_records(self, slots):
        """episode_record for several finished slots with two engine calls: every field of all
        of them is copied into ONE array per field (az_mcts_episode_records) and each record
        holds views of its episode's rows."""
        n = len(slots)
        if n == 0:
            return []
        sl = np.asarray(slots, np.int32)
        moves = np.zeros(n, np.int32)
        _check(lib().az_mcts_episodes_moves(self.h, _ptr(sl), n, _ptr(moves)),
               "az_mcts_episodes_moves")
        tot = int(moves.sum())
        A, c = self.A, self.n
        width = {"C": (c, c), "A": (A,), 1: ()}
        big = {k: np.empty((tot,) + width[w], dt) for k, dt, w in self._REC}
        tg = {k: np.empty((tot,) + width[w], dt) for k, dt, w in self._TGT} if self.use_gnn else {}
        rtag = np.zeros(n, np.intc)
        rval = np.zeros(n, np.float64)
        tp = [_ptr(tg[k]) for k, _, _ in self._TGT] if self.use_gnn else [None] * 4
        _check(lib().az_mcts_episode_records(self.h, _ptr(sl), n,
                                             *[_ptr(big[k]) for k, _, _ in self._REC],
                                             _ptr(rtag), _ptr(rval), *tp),
               "az_mcts_episode_records")
        out = []
        o = 0
        vals = rval.tolist()
        for i, m in enumerate(moves.tolist()):
            r = {k: a[o:o + m] for k, a in big.items()}
            r["result"] = int(vals[i]) if rtag[i] == TAG_INT else float(vals[i])
            if tg:
                r.update({k: a[o:o + m] for k, a in tg.items()})
            out.append(r)
            o += m
        return out

    def episode_record(self, slot):
        """Per-move records of a finished episode (see include/az_mcts.h)."""
        n = _check(lib().az_mcts_episode_moves(self.h, slot), "az_mcts_episode_moves")
        A, c = self.A, self.n
        r = {"boards": np.zeros((n, c, c), np.int8), "cur": np.zeros(n, np.int8),
             "temp": np.zeros(n, np.int8), "action": np.zeros(n, np.int32),
             "pi": np.zeros((n, A), np.float64), "init_nsa": np.zeros((n, A), np.int32),
             "init_has": np.zeros((n, A), np.int8), "std_v": np.zeros(n, np.float32),
             "exp_nsa": np.zeros((n, A), np.int32), "exp_q": np.zeros((n, A), np.float64),
             "exp_tag": np.zeros((n, A), np.int8)}
        tag, val = ctypes.c_int(), ctypes.c_double()
        keys = ("boards", "cur", "temp", "action", "pi", "init_nsa", "init_has", "std_v",
                "exp_nsa", "exp_q", "exp_tag")
        _check(lib().az_mcts_episode_record(self.h, slot, *[_ptr(r[k]) for k in keys],
                                            ctypes.byref(tag), ctypes.byref(val)),
               "az_mcts_episode_record")
        r["result"] = int(val.value) if tag.value == TAG_INT else float(val.value)
        if self.use_gnn:                 # expand_tree's targets per move, computed natively
            t = {"init_policy": np.zeros((n, A), np.float64),
                 "exp_policy": np.zeros((n, A), np.float64),
                 "exp_value_tag": np.zeros(n, np.int8), "exp_value": np.zeros(n, np.float64)}
            _check(lib().az_mcts_episode_targets(
                self.h, slot, *[_ptr(t[k]) for k in ("init_policy", "exp_policy",
                                                     "exp_value_tag", "exp_value")]),
                "az_mcts_episode_targets")
            r.update(t)
        return r

    def tree_stats(self, slot):
        out = np.zeros(4, np.int64)
        _check(lib().az_mcts_tree_stats(self.h, slot, _ptr(out)), "az_mcts_tree_stats")
        return {"Es": int(out[0]), "Ns": int(out[1]), "Ps": int(out[2]), "nsa_total": int(out[3])}


def expand_result(A, init_counts, initial_value, nsa, q, tag, game=None, board=None):
    """expand_tree's return values (MCTS.py:115-146) from root statistics: init_counts
    {a: visits} before the expand searches, the root's standard value, and the root's
    (nsa, q, tag) after them."""
    initial_policy = np.zeros(A)
    for a, c in init_counts.items():
        initial_policy[a] = c
    isum = np.sum(initial_policy)
    if isum > 0:
        initial_policy = initial_policy / isum
    else:
        valids = game.getValidMoves(board, 1)
        initial_policy = valids / np.sum(valids)
    expanded_policy = np.zeros(A)
    for a in range(A):
        if tag[a] != TAG_NONE:
            expanded_policy[a] = nsa[a]
    esum = np.sum(expanded_policy)
    if esum > 0:
        expanded_policy = expanded_policy / esum
    else:
        expanded_policy = initial_policy
    expanded_value = 0
    valid_count = 0
    for a in range(A):
        if tag[a] != TAG_NONE and nsa[a] > 0:
            expanded_value += typed_q(tag[a], q[a]) * nsa[a]
            valid_count += nsa[a]
    expanded_value = expanded_value / valid_count if valid_count > 0 else initial_value
    return initial_policy, initial_value, expanded_policy, expanded_value


def _assemble_connect4(game, use_gnn, rec):
    """assemble_episode for Connect4Game with whole-episode array operations.  The objects are
    the generic path's: getSymmetries' identity comes first, so the GNN example's board is the
    canonical board itself; the mirror is np.fliplr (a view) and mirror_pi np.copy of the pi
    list (int64 for a temp-0 one-hot, float64 otherwise) with its first n entries reversed.
    Per-move objects are rows (views) of whole-episode arrays the record owns, converted to
    lists / scalars once per episode, not per move."""
    n = game.board_size
    boards = rec["boards"].astype(np.int64)
    flips = boards[:, :, ::-1]
    pis = rec["pi"]
    one_hot = (rec["temp"] == 0).tolist()
    mirror_f = pis.copy()
    mirror_f[:, :n] = pis[:, n - 1::-1]
    mirror_i = mirror_f.astype(np.int64)
    pl_f, pl_i = pis.tolist(), pis.astype(np.int64).tolist()
    curs = rec["cur"].tolist()
    r = rec["result"]
    last = -int(curs[-1])
    signs = [r * ((-1) ** (c != last)) for c in curs]
    std = []
    for i, sg in enumerate(signs):
        if one_hot[i]:
            std.append((boards[i], pl_i[i], sg))
            std.append((flips[i], mirror_i[i], sg))
        else:
            std.append((boards[i], pl_f[i], sg))
            std.append((flips[i], mirror_f[i], sg))
    if not use_gnn:
        return std, []
    ip, ep = rec["init_policy"], rec["exp_policy"]      # arrays of this record alone
    sv = rec["std_v"]                                   # float32: sv[i] is an np.float32
    tags, vals = rec["exp_value_tag"], rec["exp_value"]
    v32 = vals.astype(np.float32)
    ev = [typed_q(t, v) if t != TAG_F32 else v32[i]
          for i, (t, v) in enumerate(zip(tags.tolist(), vals.tolist()))]
    gnn = [(boards[i], c, ip[i], sv[i], ep[i], ev[i], signs[i]) for i, c in enumerate(curs)]
    return std, gnn


def assemble_episode(game, args, rec):
    """Coach.executeEpisode's examples (Coach.py:27-79, the same steps as Coach.episode_g)
    from an engine episode record."""
    use_gnn = bool(args.get("use_gnn", False) if isinstance(args, dict)
                   else getattr(args, "use_gnn", False))
    if type(game).__name__ == "Connect4Game" and (not use_gnn or "init_policy" in rec):
        return _assemble_connect4(game, use_gnn, rec)
    A = game.getActionSize()
    examples, gnn_examples = [], []
    for i in range(len(rec["cur"])):
        canonical = rec["boards"][i].astype(np.int64)
        cur = int(rec["cur"][i])
        if rec["temp"][i] == 0:
            pi = [int(x) for x in rec["pi"][i]]
        else:
            pi = rec["pi"][i].tolist()
        sym = game.getSymmetries(canonical, pi)
        examples.extend([b, cur, p, None] for b, p in sym)
        if use_gnn:
            s = game.stringRepresentation(canonical)
            if "init_policy" in rec:     # az_mcts_episode_targets (same values and types)
                res = (rec["init_policy"][i].copy(), np.float32(rec["std_v"][i]),
                       rec["exp_policy"][i].copy(),
                       typed_q(int(rec["exp_value_tag"][i]), rec["exp_value"][i]))
            else:
                init_counts = {a: int(rec["init_nsa"][i][a]) for a in range(A)
                               if rec["init_has"][i][a] != TAG_NONE}
                res = expand_result(A, init_counts, np.float32(rec["std_v"][i]),
                                    rec["exp_nsa"][i].tolist(), rec["exp_q"][i].tolist(),
                                    rec["exp_tag"][i].tolist(), game, canonical)
            for b, _ in sym:
                if game.stringRepresentation(b) == s:
                    gnn_examples.append([b, cur, *res, None])
                    break
    r = rec["result"]
    cur = -int(rec["cur"][-1])

    def sign(p):
        return r * ((-1) ** (p != cur))
    std = [(x[0], x[2], sign(x[1])) for x in examples]
    if use_gnn and gnn_examples:
        return std, [(x[0], x[1], x[2], x[3], x[4], x[5], sign(x[1])) for x in gnn_examples]
    return std, []


class NativeMCTS:
    """One slot of an Engine with the reference MCTS's root-level logic (MCTS.py:29-149)."""

    def __init__(self, engine, slot, game, args, rng=None):
        self.engine, self.slot, self.game, self.args = engine, slot, game, args
        self.rng = rng

    def _choice(self, *a, **k):
        return (np.random if self.rng is None else self.rng).choice(*a, **k)

    def _root(self, board):
        nsa, q, tag = self.engine.root_edges(self.slot, board)
        return nsa, q, tag

    def getActionProb_g(self, canonicalBoard, temp=1):
        """MCTS.py:29-58 (the searches run in the engine)."""
        self.engine.clear_predictions(self.slot)
        yield ("search", canonicalBoard, self.args.numMCTSSims)
        counts = self._root(canonicalBoard)[0]
        if temp == 0:
            best = np.array(np.argwhere(counts == np.max(counts))).flatten()
            a = self._choice(best)
            probs = [0] * len(counts)
            probs[a] = 1
            return probs
        counts = [(x + EPS) ** (1. / temp) for x in counts]
        total = float(sum(counts))
        if total <= 0:
            valids = self.game.getValidMoves(canonicalBoard, 1)
            if np.sum(valids) > 0:
                return valids / np.sum(valids)
            return np.ones(len(counts)) / len(counts)
        return [x / total for x in counts]

    def expand_tree_g(self, canonicalBoard, expand_by=5):
        """MCTS.py:60-149."""
        s = self.game.stringRepresentation(canonicalBoard)
        A = self.game.getActionSize()

        def root_visits():
            nsa, _, tag = self._root(canonicalBoard)
            return {a: nsa[a] for a in range(A) if tag[a] != TAG_NONE}

        initial_counts = root_visits()
        if not initial_counts:
            yield ("search", canonicalBoard, self.args.numMCTSSims)
            initial_counts = root_visits()
        std_v = self.engine.get_std(self.slot, canonicalBoard)
        if std_v is None:
            _, std_v = yield ("predict", canonicalBoard)
            self.engine.set_std(self.slot, canonicalBoard, std_v)
        initial_value = np.float32(std_v)
        yield ("search", canonicalBoard, expand_by)
        nsa, q, tag = self._root(canonicalBoard)
        res = expand_result(A, initial_counts, initial_value, nsa, q, tag, self.game,
                            canonicalBoard)
        return {s: res}


class ArenaPlayer:
    """An Arena action function, the reference's `lambda x: np.argmax(mcts.getActionProb(x,
    temp=0))` (Coach.py:140-142), with the searches in a one-slot native engine.  The tree
    persists across moves and games exactly like the reference's MCTS object, which is created
    once per iteration and reused for the whole arena -- so arena games depend on each other
    and are played one after the other; what moves native is the per-simulation search and
    rules work (MCTS.py:151-240).  Leaves go to the network one at a time (`predict_both` on
    one board when use_gnn, else `predict_batch`), as the reference's batch-1 calls.

    Speculative leaf batches (nets whose rows are batch-invariant, `batch_invariant_rows`): a
    leaf the search asks for is evaluated together with the non-terminal boards one move below
    it (at most batch_invariant_rows - 1 of them, skipping boards already expanded or cached),
    and the children's rows go into the engine's row cache (az_mcts_collect_spec /
    az_mcts_feed_spec), so a later simulation that reaches one of them as a new leaf is expanded
    inside the engine without a network call or a return to Python.  The rows of
    such a batch are bit-identical to batch-1 evaluations of the same boards
    (tests/test_gpu_selfplay.py), so the search -- and every arena game -- is unchanged; only the
    number of launches drops.  The cache lives as long as the player (one arena: the network
    does not change)."""

    def __init__(self, game, nnet, args, prefetch=True):
        get = (lambda k, d=None: args.get(k, d)) if isinstance(args, dict) else \
            (lambda k, d=None: getattr(args, k, d))
        self.use_gnn = bool(get("use_gnn", False))
        self.nnet, self.args = nnet, args
        self.eng = Engine(game, 1, float(get("cpuct", 1.0)), self.use_gnn)
        self.mcts = NativeMCTS(self.eng, 0, game, args)
        rows = int(getattr(nnet, "batch_invariant_rows", 0) or 0) if prefetch else 0
        self.spec = rows if rows >= 2 else 0
        self.calls = 0
        if self.spec:
            self._batch = np.zeros((self.spec, self.eng.n, self.eng.n), np.int8)
            self._pbatch = _ptr(self._batch)

    @property
    def hits(self):
        """Leaves the search expanded from speculative rows (no network call of their own)."""
        return self.eng.cache_stats()[1]

    def _search(self, board, sims):
        self.eng.begin(0, board, sims)
        try:
            self._search_loop()
        except BaseException:
            self.eng.abandon(0)     # a raise mid-search (AZ_STRICT_NN) leaves the slot reusable
            raise

    def _search_loop(self):
        if self.spec:
            self._search_spec()
            return
        from selfplay import _net_call
        idle = 0
        while self.eng.remaining(0) > 0:
            k = self.eng.collect(1)
            if k == 0:
                idle += 1
                if idle > 4:
                    raise RuntimeError("native arena search made no progress")
                continue
            idle = 0
            self.calls += 1
            try:
                pi, v, gpi, gv = _net_call(self.nnet, self.eng.leaf_boards[:k], self.use_gnn)
            except Exception as ex:  # MCTS.py:195-200: uniform priors, value 0 (counted)
                self.eng.feed(k, failed=True)      # engine first: left consistent if
                nn_fallback.record("ArenaPlayer", ex, k)   # AZ_STRICT_NN raises here
                continue
            self.eng.feed(k, pi, v, gpi, gv)

    def _search_spec(self):
        """The search loop with speculative leaf batches: the engine hands out the leaf and its
        children in one buffer and takes all their rows back (az_mcts_collect_spec /
        az_mcts_feed_spec); leaves found in the row cache never come back to Python."""
        from selfplay import _net_call
        eng, batch, pb, cap = self.eng, self._batch, self._pbatch, self.spec
        while True:
            k = eng.collect_spec(0, pb, cap)
            if k == 0:
                if eng.remaining(0) > 0:
                    raise RuntimeError("native arena search made no progress")
                return
            self.calls += 1
            try:
                out = _net_call(self.nnet, batch[:k], self.use_gnn)
            except Exception as ex:  # MCTS.py:195-200 for the leaf (counted), no rows kept
                eng.feed_spec(k, failed=True)
                nn_fallback.record("ArenaPlayer", ex, 1)
                continue
            eng.feed_spec(k, *out)

    def __call__(self, canonical):
        gen = self.mcts.getActionProb_g(canonical, temp=0)
        try:
            req = next(gen)
            while True:
                self._search(req[1], req[2])
                req = gen.send(None)
        except StopIteration as stop:
            return int(np.argmax(stop.value))

"""Monte-Carlo tree search, the caller of the board evaluator (reference MCTS.py:10-240).

Search statistics (Qsa, Nsa, Ns, Ps, Es, Vs) live in dicts keyed by board bytes exactly as in
the reference, and every arithmetic expression keeps the reference's operand types, so the
numeric tower (np.float32 / Python int / Python float Q values under NumPy 2 promotion) and
therefore visit counts and action choices are reproduced bit for bit given the same network
outputs and the same np.random state (tests/test_mcts_golden.py).

The descent is iterative (path recorded, then backed up) instead of recursive; the reference's
sign convention is kept: a new leaf or a terminal state hands its value UN-negated to its
parent, and every interior node updates with the value it receives and passes on its negation
(MCTS.py:154-157,190-193,226-240).

Every search routine is written once, as a generator (`*_g`) that YIELDS a leaf-evaluation
request `(board, want_gnn)` and receives `(std, gnn, err)` back: std/gnn are `(pi, v)` pairs or
None, err the exception a failed evaluation raised.  The reference-shaped methods
(`search`, `getActionProb`, `expand_tree`) drive that generator with batch-1 `predict` /
`predict_with_gnn` calls; selfplay.py drives many of them in lock step with one batched
`predict_both` launch per simulation.  Same code either way, so the lock-step driver inherits
the search parity.
"""
import logging
import math

import numpy as np

import nn_fallback

EPS = 1e-8

log = logging.getLogger(__name__)


class MCTS:
    def __init__(self, game, nnet, args, rng=None):
        self.game = game
        self.nnet = nnet
        self.args = args
        self.rng = rng            # None: the global np.random stream, as the reference
        self.Qsa = {}
        self.Nsa = {}
        self.Ns = {}
        self.Ps = {}
        self.Es = {}
        self.Vs = {}
        self.standard_predictions = {}
        self.gnn_predictions = {}
        self.expanded = False
        self.expanded_nodes = {}

    def _use_gnn(self):
        return bool(getattr(self.args, "use_gnn", False)) if not isinstance(self.args, dict) \
            else bool(self.args.get("use_gnn", False))

    def _choice(self, *a, **k):
        return (np.random if self.rng is None else self.rng).choice(*a, **k)

    # ------------------------------------------------------------------ batch-1 driver
    def evaluate_request(self, request):
        """Serve one leaf request with the reference's batch-1 calls (MCTS.py:169-174)."""
        board, want_gnn = request
        std = gnn = err = None
        try:
            std = self.nnet.predict(board)
            if want_gnn:
                gnn = self.nnet.predict_with_gnn(board)
        except Exception as e:  # handled where the reference handles it (search / expand_tree)
            err = e
        return std, gnn, err

    def drive(self, gen):
        """Run a search generator to completion with batch-1 network calls."""
        try:
            request = next(gen)
            while True:
                request = gen.send(self.evaluate_request(request))
        except StopIteration as stop:
            return stop.value

    def getActionProb(self, canonicalBoard, temp=1):
        return self.drive(self.getActionProb_g(canonicalBoard, temp))

    def expand_tree(self, canonicalBoard, expand_by=5):
        return self.drive(self.expand_tree_g(canonicalBoard, expand_by))

    def search(self, canonicalBoard, expansion=False):
        return self.drive(self.search_g(canonicalBoard, expansion))

    # ------------------------------------------------------------------ root policies
    def _root_counts(self, s):
        return [self.Nsa[(s, a)] if (s, a) in self.Nsa else 0
                for a in range(self.game.getActionSize())]

    def getActionProb_g(self, canonicalBoard, temp=1):
        """MCTS.py:29-58: numMCTSSims searches, then visit counts -> policy (temp 0: argmax
        with a np.random.choice tie-break)."""
        self.standard_predictions = {}
        self.gnn_predictions = {}
        for _ in range(self.args.numMCTSSims):
            yield from self.search_g(canonicalBoard)
        counts = self._root_counts(self.game.stringRepresentation(canonicalBoard))
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
        """MCTS.py:60-149: extra searches from the root; returns
        {root: (initial_pi, initial_v, expanded_pi, expanded_v)} for GNN training targets."""
        s = self.game.stringRepresentation(canonicalBoard)
        A = self.game.getActionSize()
        self.expanded = True
        self.expanded_nodes = {}

        def root_visits():
            return {a: n for (k, a), n in self.Nsa.items() if k == s}

        initial_counts = root_visits()
        if not initial_counts:
            for _ in range(self.args.numMCTSSims):
                yield from self.search_g(canonicalBoard)
            initial_counts = root_visits()
        initial_policy = np.zeros(A)
        for a, c in initial_counts.items():
            initial_policy[a] = c
        isum = np.sum(initial_policy)
        if isum > 0:
            initial_policy = initial_policy / isum
        else:
            valids = self.game.getValidMoves(canonicalBoard, 1)
            initial_policy = valids / np.sum(valids)

        if s not in self.standard_predictions:
            std, _, err = yield (canonicalBoard, False)    # unguarded in the reference (:108-113)
            if std is None:
                raise err
            std_pi, std_v = std
            self.standard_predictions[s] = (std_pi, std_v)
        initial_value = self.standard_predictions[s][1]

        for _ in range(expand_by):
            yield from self.search_g(canonicalBoard)

        expanded_policy = np.zeros(A)
        for a, c in root_visits().items():
            expanded_policy[a] = c
        esum = np.sum(expanded_policy)
        if esum > 0:
            expanded_policy = expanded_policy / esum
        else:
            expanded_policy = initial_policy

        expanded_value = 0
        valid_count = 0
        for a in range(A):
            if (s, a) in self.Qsa and (s, a) in self.Nsa and self.Nsa[(s, a)] > 0:
                expanded_value += self.Qsa[(s, a)] * self.Nsa[(s, a)]
                valid_count += self.Nsa[(s, a)]
        expanded_value = expanded_value / valid_count if valid_count > 0 else initial_value

        self.expanded_nodes[s] = (initial_policy, initial_value, expanded_policy, expanded_value)
        self.expanded = False
        return self.expanded_nodes

    # ------------------------------------------------------------------ search
    def _evaluate_leaf_g(self, s, board):
        """New leaf: NN priors masked by the valid moves and renormalised; returns the leaf
        value (MCTS.py:162-200).  Network errors degrade to uniform priors and value 0."""
        if s not in self.Vs:
            self.Vs[s] = self.game.getValidMoves(board, 1)
        valids = self.Vs[s]
        use_gnn = self._use_gnn()
        std, gnn, err = yield (board, use_gnn)
        try:
            if std is None:
                raise err
            std_pi, std_v = std
            self.standard_predictions[s] = (std_pi, std_v)
            if use_gnn:
                if gnn is None:
                    raise err
                gnn_pi, gnn_v = gnn
                self.gnn_predictions[s] = (gnn_pi, gnn_v)
                self.Ps[s] = gnn_pi
            else:
                self.Ps[s] = std_pi
            self.Ps[s] = self.Ps[s] * valids
            total = np.sum(self.Ps[s])
            if total > 0:
                self.Ps[s] /= total
            else:
                log.warning("All valid moves were masked, using uniform policy")
                self.Ps[s] = valids / np.sum(valids)
            self.Ns[s] = 0
            if self._use_gnn() and s in self.gnn_predictions:
                return self.gnn_predictions[s][1]
            return self.standard_predictions[s][1]
        except Exception as e:  # the reference's degradation (MCTS.py:195-200), counted
            nn_fallback.record("MCTS.search", e)
            self.Ps[s] = valids / np.sum(valids)
            self.Ns[s] = 0
            return 0

    def _select(self, s):
        """UCB argmax over valid actions (MCTS.py:202-218); -1 when none."""
        valids = self.Vs[s]
        P = self.Ps[s]
        cpuct = self.args.cpuct
        best_u, best_a = -float("inf"), -1
        for a in range(self.game.getActionSize()):
            if not valids[a]:
                continue
            if (s, a) in self.Qsa:
                u = self.Qsa[(s, a)] + cpuct * P[a] * math.sqrt(self.Ns[s]) / (1 + self.Nsa[(s, a)])
            else:
                u = cpuct * P[a] * math.sqrt(self.Ns[s] + EPS)
            if u > best_u:
                best_u, best_a = u, a
        return best_a

    def search_g(self, canonicalBoard, expansion=False):
        path = []                     # (s, a) edges taken from the root
        board = canonicalBoard
        two_player = bool(getattr(self.game, "is_two_player", False))
        while True:
            s = self.game.stringRepresentation(board)
            if s not in self.Es:
                self.Es[s] = self.game.getGameEnded(board, 1)
            if self.Es[s] != 0:
                v = self.Es[s]
                break
            if expansion and self.Ns.get(s, 0) >= self.args.numMCTSSims:
                v = 0
                break
            if s not in self.Ps:
                v = yield from self._evaluate_leaf_g(s, board)
                break
            a = self._select(s)
            if a == -1:
                v = 0
                break
            path.append((s, a))
            nxt, player = self.game.getNextState(board, 1, a)
            board = self.game.getCanonicalForm(nxt, player)
        # back-up: each interior node takes the value its child returned and returns -v
        # (or v for a single-player game)
        for s, a in reversed(path):
            if (s, a) in self.Qsa:
                self.Qsa[(s, a)] = (self.Nsa[(s, a)] * self.Qsa[(s, a)] + v) / (self.Nsa[(s, a)] + 1)
                self.Nsa[(s, a)] += 1
            else:
                self.Qsa[(s, a)] = v
                self.Nsa[(s, a)] = 1
            self.Ns[s] += 1
            v = -v if two_player else v
        return v

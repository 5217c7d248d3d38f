"""Capture golden vectors from the reference (andrpac/alphazero-gnn) on CPU.

Run ONLY in the build container, where the read-only reference is mounted:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py [--only NAME ...]

The reference is imported from /root/reference (nothing is written there) and exercised
through its own public entry points; intermediates are taken with forward hooks, never by
re-deriving them.  Only data (inputs + outputs) is written to tests/golden/.  Nothing in
tests/, bench.py or __graft_entry__.py reads /root/reference at run time.

Fixtures:
  G1 c4_net.npz          Connect4Net torch-default weights (seed 0), 256 boards, predict + batched fwd
  G2 c4_gnn.npz          Connect4 GNN (synthetic PCG64 weights, seed 1234): predict_with_gnn on 64
                         boards + one 64-row star forward (alpha, agg, row-0 per layer, heads)
  G2t c4_gnn_trained_lr01.npz / _lr001.npz: the same net after 2 reference train() calls at
                         lr 0.01 / 5 at lr 0.001 (dropout 0):
                         examples, trained CNN, GNN checksums, predict / predict_with_gnn (pi, v,
                         log pi) on 1,576 boards
  G3 synth_gnn.npz      PolicyValueGNN(64): per-destination 32x32 grid forward + literal star N=4096
  G4 ttt3.npz            TicTacToe 3x3 CNN+GNN weights (seed 0), predict/predict_with_gnn on every
                         reachable canonical position
  G4b ttt4.npz           TicTacToe 4x4 (the YAML default; F = 512, A = 17): PCG64 weights,
                         predict/predict_with_gnn on 2,000 random-play positions, one train()
  G5 train_ttt3.npz      one TicTacToeGNNWrapper.train (2 epochs) -> params after Adam
     train_c4.npz        one Connect4GNNWrapper.train (dropout 0, 2 epochs) -> CNN params + GNN checksums
  G6 mcts_c4.npz/json    Connect4 self-play episodes (sims 25, no GNN): per-move root counts/pi/choices,
                         every NN output the search requested, the examples
     mcts_ttt3.npz/json  TicTacToe 3x3 GNN self-play episodes with expand_tree
     mcts_c4_gnn.npz/json  Connect4 GNN self-play at the north-star setting (sims 100, use_gnn,
                         expand_tree; G1 CNN weights + G2 GNN weights), episodes 0-2
     mcts_c4_gnn_trace.npz G6c: the same setting, episodes 0-15: every UCB selection of the
                         reference's search (state crc32, action, score gap, Ns) + the examples
  G7 coach_ttt3.json     one full TicTacToe 3x3 GNN Coach iteration (seeds 0): counts, arena W/L/D
  G8 rules.npz           game rules on random-play positions (Connect4 n=7,5; TicTacToe n=3,4):
                         getGameEnded for both players, getValidMoves, every legal next state,
                         getSymmetries boards and policies
  G9 resume_ttt3/        --load_model resume (main.py:259-280, Coach.py:187-201): the checkpoint
                         (best_gnn.pth.tar) and example history (best_gnn.pth.tar.examples) the
                         reference wrote after one TicTacToe 3x3 GNN iteration (G7's run), and
                         resume_ttt3.json: what the reference's resumed iteration did (seeds 1)
"""
import argparse
import importlib.util
import json
import os
import random
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)

from gnn_utils import PolicyValueGNN  # noqa: E402
from connect4.Connect4Game import Connect4Game  # noqa: E402
from connect4.Connect4Net import Connect4NNetWrapper  # noqa: E402
from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402
from tictactoe.TicTacToeGame import TicTacToeGame  # noqa: E402
from tictactoe.TicTacToeGNN import TicTacToeGNNWrapper  # noqa: E402
import MCTS as ref_mcts  # noqa: E402
import Coach as ref_coach  # noqa: E402
import Arena as ref_arena  # noqa: E402

_spec = importlib.util.spec_from_file_location(
    "az_weights", os.path.join(REPO, "alphazero-gnn_amd", "azhip", "weights.py"))
W = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(W)

torch.set_num_threads(8)


class dotdict(dict):
    """Same semantics as main.py:18-23."""
    def __getattr__(self, name):
        return self[name]

    def __setattr__(self, name, value):
        self[name] = value


def base_args(**kw):
    a = dotdict(lr=0.001, dropout=0.3, epochs=20, batch_size=64, use_gnn=False, gnn_layers=2,
                numIters=1, numEps=20, tempThreshold=15, updateThreshold=0.6,
                maxlenOfQueue=200000, numItersForTrainExamplesHistory=5,
                numMCTSSims=10, cpuct=1.0, expand_by=5, arenaCompare=100)
    a.update(kw)
    return a


def sd_np(module):
    return {k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def out(name):
    return os.path.join(HERE, name)


def random_play_boards(game, n, rng, max_moves=48):
    """Canonical boards reached by uniformly random legal play (seeded)."""
    boards = []
    while len(boards) < n:
        b = game.getInitBoard()
        p = 1
        steps = int(rng.integers(0, max_moves))
        for _ in range(steps):
            if game.getGameEnded(b, p) != 0:
                break
            v = game.getValidMoves(game.getCanonicalForm(b, p), 1)
            a = int(rng.choice(np.flatnonzero(v)))
            b, p = game.getNextState(b, p, a)
        boards.append(game.getCanonicalForm(b, p).astype(np.int8))
    return np.stack(boards)


# ----------------------------------------------------------------------------------- G1
def g1():
    torch.manual_seed(0)
    np.random.seed(0)
    game = Connect4Game(7)
    net = Connect4NNetWrapper(game, base_args())
    sd = sd_np(net.nnet)
    rng0 = np.random.default_rng(0)
    rnd = rng0.integers(-1, 2, size=(128, 7, 7)).astype(np.int8)
    play = random_play_boards(game, 128, np.random.default_rng(1))
    boards = np.concatenate([rnd, play])
    pis, vs = [], []
    for b in boards:
        pi, v = net.predict(b.astype(np.int64))
        pis.append(pi)
        vs.append(v)
    net.nnet.eval()
    with torch.no_grad():
        lp, vb = net.nnet(torch.FloatTensor(boards.astype(np.float64)))
    np.savez(out("c4_net.npz"), boards=boards, pi_b1=np.stack(pis).astype(np.float32),
             v_b1=np.array(vs, np.float32), logp_batch=lp.numpy(), v_batch=vb.numpy()[:, 0],
             **{"w/" + k: v for k, v in sd.items()})
    return net, boards


# ----------------------------------------------------------------------------------- G2
GNN_C4_SEED = 1234


def g2(c4net_sd, boards):
    game = Connect4Game(7)
    torch.manual_seed(0)
    g = Connect4GNNWrapper(game, base_args(use_gnn=True))
    g.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in c4net_sd.items()})
    t0 = time.time()
    gsd = W.synthetic_state_dict(W.gnn_spec(3136, 2), GNN_C4_SEED)
    g.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
    del gsd
    print(f"  G2 weights generated+loaded in {time.time() - t0:.1f}s")
    sel = boards[::4][:64]
    pis, vs = [], []
    for b in sel:
        pi, v = g.predict_with_gnn(b.astype(np.int64))
        pis.append(pi)
        vs.append(v)
    # one 64-row star forward (the training-time shape, Connect4GNN.py:178-184) in eval mode
    g.nnet.eval()
    g.gnn.eval()
    rec = {"attn": [[], []], "comb": [None, None], "row0": [None, None]}
    hooks = []
    for li, layer in enumerate(g.gnn.layers):
        hooks.append(layer.attention.register_forward_hook(
            lambda m, i, o, li=li: rec["attn"][li].append(torch.sigmoid(o).item())))
        hooks.append(layer.gate.register_forward_hook(
            lambda m, i, o, li=li: rec["comb"].__setitem__(li, i[0].detach().clone())))
        hooks.append(layer.register_forward_hook(
            lambda m, i, o, li=li: rec["row0"].__setitem__(li, o[0].detach().clone())))
    with torch.no_grad():
        feats = g.extract_features(torch.FloatTensor(sel.astype(np.float64)))
        enh = g.gnn(feats)
        lp, v = g.apply_policy_value_heads(enh)
    for h in hooks:
        h.remove()
    F = 3136
    np.savez(out("c4_gnn.npz"), seed=np.int64(GNN_C4_SEED), boards=sel,
             pi_gnn_b1=np.stack(pis).astype(np.float32), v_gnn_b1=np.array(vs, np.float32),
             star_alpha_raw=np.array(rec["attn"], np.float32),
             star_agg=np.stack([c[0, F:].numpy() for c in rec["comb"]]),
             star_row0=np.stack([r.numpy() for r in rec["row0"]]),
             star_enh_row0=enh[0].numpy(), star_enh_rowsum=enh.sum(1).numpy(),
             star_logp=lp.numpy(), star_v=v.numpy()[:, 0])
    return g


# ----------------------------------------------------------------------------------- G3
SYN_SEED_W, SYN_SEED_X, SYN_SEED_STAR = 64, 0, 5


def grid_csr(h, w):
    """4-neighbour grid, CSR by destination, sources ascending."""
    rowptr = [0]
    col = []
    for r in range(h):
        for c in range(w):
            nb = []
            for dr, dc in ((-1, 0), (0, -1), (0, 1), (1, 0)):
                rr, cc = r + dr, c + dc
                if 0 <= rr < h and 0 <= cc < w:
                    nb.append(rr * w + cc)
            col += sorted(nb)
            rowptr.append(len(col))
    return np.array(rowptr, np.int32), np.array(col, np.int32)


def g3():
    gnn = PolicyValueGNN(64, 2)
    sd = W.synthetic_state_dict(W.gnn_spec(64, 2), SYN_SEED_W)
    gnn.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gnn.eval()
    rowptr, col = grid_csr(32, 32)
    rng = np.random.Generator(np.random.PCG64(SYN_SEED_X))
    x0 = (rng.random((1024, 64), dtype=np.float32) * np.float32(2) - np.float32(1))
    xs = [torch.from_numpy(x0)]
    with torch.no_grad():
        for layer in gnn.layers:
            cur = xs[-1]
            nxt = torch.empty_like(cur)
            for d in range(1024):
                nb = col[rowptr[d]:rowptr[d + 1]]
                feats = torch.cat([cur[d:d + 1], cur[torch.from_numpy(nb.astype(np.int64))]])
                nxt[d] = layer(feats)[0]
            xs.append(nxt)
        grid_out = gnn.output_transform(xs[-1])
        rng2 = np.random.Generator(np.random.PCG64(SYN_SEED_STAR))
        star_x = rng2.random((4096, 64), dtype=np.float32) * np.float32(2) - np.float32(1)
        star_out = gnn(torch.from_numpy(star_x))
    np.savez(out("synth_gnn.npz"), seed_w=np.int64(SYN_SEED_W), seed_x=np.int64(SYN_SEED_X),
             seed_star=np.int64(SYN_SEED_STAR), rowptr=rowptr, col=col,
             grid_x1=xs[1].numpy(), grid_x2=xs[2].numpy(), grid_out=grid_out.numpy(),
             star_out_head=star_out[:65].numpy(), star_out_rowsum=star_out.sum(1).numpy())


# ----------------------------------------------------------------------------------- G4
def reachable_ttt(game):
    """Every distinct canonical board reachable from the empty board (BFS)."""
    seen = {}
    frontier = [(game.getInitBoard(), 1)]
    while frontier:
        nxt = []
        for b, p in frontier:
            c = game.getCanonicalForm(b, p)
            key = c.tobytes()
            if key in seen:
                continue
            seen[key] = c
            if game.getGameEnded(b, p) != 0:
                continue
            v = game.getValidMoves(c, 1)
            for a in np.flatnonzero(v):
                nb, np_ = game.getNextState(b, p, int(a))
                nxt.append((nb, np_))
        frontier = nxt
    return np.stack([seen[k] for k in sorted(seen)]).astype(np.int8)


def g4():
    torch.manual_seed(0)
    game = TicTacToeGame(3)
    net = TicTacToeGNNWrapper(game, base_args(use_gnn=True))
    sd = sd_np(net.nnet)
    gsd = sd_np(net.gnn)
    boards = reachable_ttt(game)
    pis, vs, gpis, gvs = [], [], [], []
    for b in boards:
        pi, v = net.predict(b.astype(np.int64))
        gpi, gv = net.predict_with_gnn(b.astype(np.int64))
        pis.append(pi)
        vs.append(v)
        gpis.append(gpi)
        gvs.append(gv)
    np.savez(out("ttt3.npz"), boards=boards, pi=np.stack(pis), v=np.array(vs, np.float32),
             pi_gnn=np.stack(gpis), v_gnn=np.array(gvs, np.float32),
             **{"w/" + k: v for k, v in sd.items()}, **{"g/" + k: v for k, v in gsd.items()})
    return net, boards


# ----------------------------------------------------------------------------------- G5
def make_examples(boards, action_size, n, ngnn, rng):
    idx = rng.integers(0, len(boards), n)
    pis = rng.dirichlet(np.ones(action_size), n).astype(np.float64)
    zs = rng.choice([-1, 1, 1e-4], n)
    ex = [(boards[i].astype(np.int64), pis[j], zs[j]) for j, i in enumerate(idx)]
    gidx = rng.integers(0, len(boards), ngnn)
    gex = []
    for j, i in enumerate(gidx):
        ipi = rng.dirichlet(np.ones(action_size)).astype(np.float64)
        epi = rng.dirichlet(np.ones(action_size)).astype(np.float64)
        gex.append((boards[i].astype(np.int64), 1, ipi, np.float32(rng.uniform(-1, 1)), epi,
                    np.float32(rng.uniform(-1, 1)), 1))
    return ex, gex


def pack_examples(ex, gex):
    return dict(ex_boards=np.stack([e[0] for e in ex]).astype(np.int8),
                ex_pis=np.stack([e[1] for e in ex]), ex_z=np.array([e[2] for e in ex], np.float64),
                gex_boards=np.stack([e[0] for e in gex]).astype(np.int8),
                gex_epis=np.stack([e[4] for e in gex]),
                gex_ev=np.array([e[5] for e in gex], np.float32))


CHECK_IDX = 97  # fixed flat indices for GNN param spot checks: PCG64(CHECK_IDX)


def g5(ttt_boards, c4net_sd, c4_boards):
    # --- TicTacToe 3x3: deterministic (no dropout anywhere, TicTacToeNet.py:28-48)
    torch.manual_seed(0)
    game = TicTacToeGame(3)
    net = TicTacToeGNNWrapper(game, base_args(use_gnn=True, epochs=2))
    ex, gex = make_examples(ttt_boards, 10, 200, 100, np.random.default_rng(11))
    np.random.seed(7)
    net.train(ex, gex)
    np.savez(out("train_ttt3.npz"), np_seed=np.int64(7), epochs=np.int64(2),
             **pack_examples(ex, gex),
             **{"w/" + k: v for k, v in sd_np(net.nnet).items()},
             **{"g/" + k: v for k, v in sd_np(net.gnn).items()})
    # --- Connect4 with dropout 0 (Connect4Net.py:28): CNN params in full, GNN by checksums
    game = Connect4Game(7)
    g = Connect4GNNWrapper(game, base_args(use_gnn=True, epochs=2, dropout=0.0))
    g.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in c4net_sd.items()})
    gsd = W.synthetic_state_dict(W.gnn_spec(3136, 2), GNN_C4_SEED)
    g.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
    del gsd
    ex, gex = make_examples(c4_boards, 8, 100, 64, np.random.default_rng(12))
    np.random.seed(9)
    t0 = time.time()
    g.train(ex, gex)
    print(f"  G5 c4 train {time.time() - t0:.1f}s")
    rng = np.random.Generator(np.random.PCG64(CHECK_IDX))
    chk = {}
    for k, v in g.gnn.state_dict().items():
        a = v.numpy().ravel()
        ii = rng.integers(0, a.size, 64)
        chk["gsum/" + k] = np.float64(a.astype(np.float64).sum())
        chk["gabs/" + k] = np.float64(np.abs(a.astype(np.float64)).sum())
        chk["gidx/" + k] = ii
        chk["gval/" + k] = a[ii]
    np.savez(out("train_c4.npz"), np_seed=np.int64(9), epochs=np.int64(2),
             gnn_seed=np.int64(GNN_C4_SEED), check_seed=np.int64(CHECK_IDX),
             **pack_examples(ex, gex), **{"w/" + k: v for k, v in sd_np(g.nnet).items()}, **chk)


def _checksums(sd, seed, full_below=0):
    """Per-tensor float64 sum / abs-sum / abs-max and 64 spot values at PCG64(seed) indices;
    tensors with fewer than `full_below` elements are stored in full ("full/<key>")."""
    rng = np.random.Generator(np.random.PCG64(seed))
    chk = {}
    for k, v in sd.items():
        a = np.asarray(v).ravel()
        ii = rng.integers(0, a.size, 64)
        chk["sum/" + k] = np.float64(a.astype(np.float64).sum())
        chk["abs/" + k] = np.float64(np.abs(a.astype(np.float64)).sum())
        chk["amax/" + k] = np.float64(np.abs(a).max())
        chk["idx/" + k] = ii
        chk["val/" + k] = a[ii]
        if a.size < full_below:
            chk["full/" + k] = np.asarray(v)
    return chk


def _both_sd(net):
    return {**{"w/" + k: v for k, v in sd_np(net.nnet).items()},
            **{"g/" + k: v for k, v in sd_np(net.gnn).items()}}


def _thread_envelope(train_fn, sd_ref, threads=3):
    """Re-run a reference training with `threads` torch threads instead of 8 and return, per
    tensor, the largest |difference| to the 8-thread run and how many elements differ by more
    than 2e-5: the reference's own run-to-run spread, against which a second implementation's
    training (different summation order) is judged."""
    torch.set_num_threads(threads)
    try:
        sd = train_fn()
    finally:
        torch.set_num_threads(8)
    env = {}
    for k, v in sd_ref.items():
        e = np.abs(sd[k].astype(np.float64) - v)
        env["envmax/" + k] = np.float64(e.max())
        env["envn/" + k] = np.int64((e > 2e-5).sum())
    return env


# ---------------------------------------------------------------------------------- G2t
# (file, lr, train() calls): the reference at lr 0.01 is still finite after 2 calls and NaN
# after the 3rd (its own instability, not recorded); lr 0.001 is connect4/config.yaml's value.
G2T_RUNS = (("c4_gnn_trained_lr01.npz", 0.01, 2, True), ("c4_gnn_trained_lr001.npz", 0.001, 5, False))
# The trained output_transform weights (78.7 MB) of the runs marked True are written here,
# outside git (.gitignore) but inside the tree gpurun ships, so the GPU tests can load the
# reference's OWN trained weights: two training runs do not stay within 1e-5 of each other
# over tens of Adam steps (the step's derivative is lr / eps = 1e5-1e6 at g = 0, so fp32
# summation-order differences of 1e-10 in a near-zero gradient move a weight by ~lr).
LARGE = os.path.join(HERE, "large")


def g2t():
    for name, lr, trains, ship in G2T_RUNS:
        _g2t(name, lr, trains, tuple(range(30, 30 + trains)), ship)


def _g2t(name, lr, trains, np_seeds, ship=False):
    """Connect4 GNN after TRAINING (VERDICT r04 'do this' #1): G1's CNN + G2's GNN spec, then
    `trains` calls of the reference's Connect4GNNWrapper.train (Connect4GNN.py:122-197; 20
    epochs, dropout 0 so the run is deterministic), np.random.seed(np_seeds[t]) before call t.
    Adam moves every weight off the uniform init (|w| up to 0.24 at lr 0.01 vs the init's 0.018
    at fan_in 3136), which is what the fp16x2 GEMM split has to survive.

    Recorded: the examples, the trained CNN in full, the trained GNN as per-tensor checksums +
    spot values (479 MB: never committed), and on 1,576 boards (788 uniform {-1,0,1}, 788 reached
    by random play) the reference's batch-1 predict / predict_with_gnn (pi, v) and the per-row
    log-probabilities of predict_with_gnn's forward (Connect4GNN.py:100-112 without the exp)."""
    game = Connect4Game(7)
    z1 = np.load(out("c4_net.npz"))
    c4sd = {k[2:]: z1[k] for k in z1.files if k.startswith("w/")}
    ex, gex = make_examples(z1["boards"], 8, 200, 64, np.random.default_rng(21))

    def run():
        g = Connect4GNNWrapper(game, base_args(use_gnn=True, lr=lr, dropout=0.0))
        g.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in c4sd.items()})
        gsd = W.synthetic_state_dict(W.gnn_spec(3136, 2), GNN_C4_SEED)
        g.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
        del gsd
        for t in range(trains):
            np.random.seed(np_seeds[t])
            g.train(ex, gex)
        return g

    t0 = time.time()
    g = run()
    print(f"  G2t {name}: {trains} trains {time.time() - t0:.1f}s")
    assert all(torch.isfinite(v).all() for v in g.gnn.state_dict().values())
    env = _thread_envelope(lambda: _both_sd(run()), _both_sd(g))
    rnd = np.random.default_rng(22).integers(-1, 2, size=(788, 7, 7)).astype(np.int8)
    play = random_play_boards(game, 788, np.random.default_rng(23))
    boards = np.concatenate([rnd, play])
    pis, vs, gpis, gvs, glp = [], [], [], [], []
    g.nnet.eval()
    g.gnn.eval()
    t0 = time.time()
    for b in boards:
        pi, v = g.predict(b.astype(np.int64))
        gpi, gv = g.predict_with_gnn(b.astype(np.int64))
        with torch.no_grad():
            bt = torch.FloatTensor(b.astype(np.float64)).view(1, 7, 7)
            lp, _ = g.apply_policy_value_heads(g.gnn(g.extract_features(bt)))
        pis.append(pi)
        vs.append(v)
        gpis.append(gpi)
        gvs.append(gv)
        glp.append(lp.numpy()[0])
    print(f"  G2t {len(boards)} x (predict, predict_with_gnn) {time.time() - t0:.1f}s")
    np.savez_compressed(
        out(name), gnn_seed=np.int64(GNN_C4_SEED), lr=np.float64(lr),
        epochs=np.int64(g.args.epochs), trains=np.int64(trains),
        np_seeds=np.array(np_seeds, np.int64), check_seed=np.int64(CHECK_IDX),
        **pack_examples(ex, gex), boards=boards,
        pi_b1=np.stack(pis).astype(np.float32), v_b1=np.array(vs, np.float32),
        pi_gnn_b1=np.stack(gpis).astype(np.float32), v_gnn_b1=np.array(gvs, np.float32),
        logp_gnn_b1=np.stack(glp).astype(np.float32), **env,
        **{"w/" + k: v for k, v in sd_np(g.nnet).items()},
        **{"g" + k: v for k, v in _checksums(sd_np(g.gnn), CHECK_IDX).items()})
    if ship:
        import hashlib
        os.makedirs(LARGE, exist_ok=True)
        ot = {k: v for k, v in sd_np(g.gnn).items() if k.startswith("output_transform.")}
        np.savez(os.path.join(LARGE, name.replace(".npz", "_ot.npz")), **ot)
        digest = hashlib.sha256(b"".join(ot[k].tobytes() for k in sorted(ot))).hexdigest()
        with open(out(name.replace(".npz", "_ot.sha256")), "w") as f:
            f.write(digest + "\n")


# ---------------------------------------------------------------------------------- G4b
TTT4_SEED_CNN, TTT4_SEED_GNN = 41, 42


def g4b():
    """TicTacToe 4x4, the default of tictactoe/config.yaml:5 (VERDICT r04 'do this' #3):
    conv3 without padding gives F = 128 * 2 * 2 = 512 and A = 17 (TicTacToeNet.py:16-26,
    TicTacToeGNN.py:14).  Weights from the documented PCG64 generator (CNN seed 41, GNN seed 42;
    the GNN is 13.6 MB, never committed).  2,000 positions reached by seeded random play, the
    reference's batch-1 predict and predict_with_gnn on each, then one train() (2 epochs, the
    YAML's lr 0.001; TicTacToe has no dropout, so it is deterministic) with every parameter
    recorded as checksums + spot values, the CNN and the GNN's small tensors in full."""
    game = TicTacToeGame(4)

    def make():
        net = TicTacToeGNNWrapper(game, base_args(use_gnn=True, epochs=2))
        csd = W.synthetic_state_dict(W.tictactoe_net_spec(4), TTT4_SEED_CNN)
        gsd = W.synthetic_state_dict(W.gnn_spec(512, 2), TTT4_SEED_GNN)
        net.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in csd.items()})
        net.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
        return net

    net = make()
    boards = random_play_boards(game, 2000, np.random.default_rng(43), max_moves=17)
    pis, vs, gpis, gvs = [], [], [], []
    t0 = time.time()
    for b in boards:
        pi, v = net.predict(b.astype(np.int64))
        gpi, gv = net.predict_with_gnn(b.astype(np.int64))
        pis.append(pi)
        vs.append(v)
        gpis.append(gpi)
        gvs.append(gv)
    print(f"  G4b predict {time.time() - t0:.1f}s")
    ex, gex = make_examples(boards, 17, 200, 100, np.random.default_rng(44))

    def run(net):
        np.random.seed(45)
        net.train(ex, gex)
        return net

    run(net)
    env = _thread_envelope(lambda: _both_sd(run(make())), _both_sd(net))
    np.savez_compressed(
        out("ttt4.npz"), seed_cnn=np.int64(TTT4_SEED_CNN), seed_gnn=np.int64(TTT4_SEED_GNN),
        boards=boards, pi=np.stack(pis).astype(np.float32), v=np.array(vs, np.float32),
        pi_gnn=np.stack(gpis).astype(np.float32), v_gnn=np.array(gvs, np.float32),
        np_seed=np.int64(45), epochs=np.int64(2), check_seed=np.int64(CHECK_IDX),
        **pack_examples(ex, gex), **env,
        **{"tw" + k: v for k, v in _checksums(sd_np(net.nnet), CHECK_IDX, 1 << 20).items()},
        **{"tg" + k: v for k, v in _checksums(sd_np(net.gnn), CHECK_IDX, 20000).items()})


# ----------------------------------------------------------------------------------- G6
class Recorder:
    """Transparent proxy that records every NN output the search requests."""

    def __init__(self, net):
        self.net = net
        self.std = {}
        self.gnn = {}

    def predict(self, board):
        pi, v = self.net.predict(board)
        self.std[board.tobytes()] = (board.astype(np.int8).copy(), np.array(pi), np.float32(v))
        return pi, v

    def predict_with_gnn(self, board):
        pi, v = self.net.predict_with_gnn(board)
        self.gnn[board.tobytes()] = (board.astype(np.int8).copy(), np.array(pi), np.float32(v))
        return pi, v


def _tag(x):
    if isinstance(x, np.floating):
        return "np." + x.dtype.name
    return type(x).__name__


def run_episodes(game, net, args, episodes, name, n, compress=False):
    coach = ref_coach.Coach.__new__(ref_coach.Coach)  # skip pnet construction (Coach.py:21)
    coach.game, coach.args = game, args
    rec = Recorder(net)
    coach.nnet = rec
    moves = []
    orig_choice = np.random.choice
    choices = []

    def rec_choice(*a, **k):
        r = orig_choice(*a, **k)
        choices.append(int(r))
        return r

    results = []
    np.random.choice = rec_choice
    try:
        for e in episodes:
            np.random.seed(e)
            coach.mcts = ref_mcts.MCTS(game, rec, args)
            mc = coach.mcts
            orig_gap = mc.getActionProb
            ep_moves = []

            def gap(board, temp=1, mc=mc, orig=orig_gap, ep_moves=ep_moves):
                c0 = len(choices)
                pi = orig(board, temp=temp)
                s = game.stringRepresentation(board)
                A = game.getActionSize()
                ep_moves.append(dict(
                    board=board.astype(np.int8).tolist(), temp=temp,
                    counts=[int(mc.Nsa.get((s, a), 0)) for a in range(A)],
                    q=[float(mc.Qsa[(s, a)]) if (s, a) in mc.Qsa else None for a in range(A)],
                    qtype=[_tag(mc.Qsa[(s, a)]) if (s, a) in mc.Qsa else None for a in range(A)],
                    pi=[float(x) for x in pi], choices_before=c0))
                return pi

            mc.getActionProb = gap
            c_start = len(choices)
            std_ex, gnn_ex = coach.executeEpisode()
            moves.append(ep_moves)
            results.append(dict(
                episode=e, choices=choices[c_start:],
                n_nodes=len(mc.Ns), nsa_total=int(sum(mc.Nsa.values())),
                std_examples=[(np.asarray(b).astype(int).tolist(), [float(x) for x in p], float(z))
                              for b, p, z in std_ex],
                gnn_examples=[(np.asarray(x[0]).astype(int).tolist(), int(x[1]),
                               [float(t) for t in x[2]], float(x[3]), [float(t) for t in x[4]],
                               float(x[5]), float(x[6]))
                              for x in gnn_ex]))
    finally:
        np.random.choice = orig_choice
    with open(out(name + ".json"), "w") as f:
        json.dump(dict(args=dict(args), moves=moves, episodes=results), f)
    std = list(rec.std.values())
    gnn = list(rec.gnn.values())
    (np.savez_compressed if compress else np.savez)(
             out(name + ".npz"),
             std_boards=np.stack([s[0] for s in std]).reshape(-1, n, n),
             std_pi=np.stack([s[1] for s in std]).astype(np.float32),
             std_v=np.array([s[2] for s in std], np.float32),
             gnn_boards=(np.stack([s[0] for s in gnn]).reshape(-1, n, n) if gnn
                         else np.zeros((0, n, n), np.int8)),
             gnn_pi=(np.stack([s[1] for s in gnn]).astype(np.float32) if gnn
                     else np.zeros((0, game.getActionSize()), np.float32)),
             gnn_v=np.array([s[2] for s in gnn], np.float32))


def g6(c4net, tttnet):
    run_episodes(Connect4Game(7), c4net, base_args(numMCTSSims=25), [0, 1], "mcts_c4", 7)
    run_episodes(TicTacToeGame(3), tttnet, base_args(numMCTSSims=10, use_gnn=True),
                 [0, 1, 2], "mcts_ttt3", 3)


def g6b():
    """Connect4 7x7, use_gnn, numMCTSSims 100 (the config-3 search, Coach.py:48-60 with
    expand_tree): the network is the reference's Connect4GNNWrapper with the G1 CNN weights
    (read back from c4_net.npz) and the G2 synthetic GNN weights (PCG64 seed 1234)."""
    z = np.load(out("c4_net.npz"))
    c4sd = {k[2:]: z[k] for k in z.files if k.startswith("w/")}
    game = Connect4Game(7)
    torch.manual_seed(0)
    g = Connect4GNNWrapper(game, base_args(use_gnn=True))
    g.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in c4sd.items()})
    gsd = W.synthetic_state_dict(W.gnn_spec(3136, 2), GNN_C4_SEED)
    g.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
    del gsd
    t0 = time.time()
    run_episodes(game, g, base_args(numMCTSSims=100, use_gnn=True), [0, 1, 2], "mcts_c4_gnn", 7,
                 compress=True)
    print(f"  G6b episodes {time.time() - t0:.1f}s")


def g6c(episodes=range(16)):
    """G6c mcts_c4_gnn_trace.npz: the reference's own search trace at the G6b setting (same
    network, seed = e) for episodes 0-15, for the lock-step parity test at production batch
    sizes (tests/test_gpu_selfplay.py): every UCB selection the reference's MCTS.search makes --
    crc32 of the state bytes, the chosen action, the best-minus-second score gap and Ns[s] -- and
    the episode's std / GNN examples.  The selection is inline in MCTS.search (MCTS.py:202-218),
    so it is read from inside the reference's own frame when search calls game.getNextState
    right after choosing (MCTS.py:223): the scores are recomputed there from the same Qsa / Ps /
    Ns / Nsa with the same float expressions."""
    import math
    import zlib
    z = np.load(out("c4_net.npz"))
    c4sd = {k[2:]: z[k] for k in z.files if k.startswith("w/")}
    game = Connect4Game(7)
    torch.manual_seed(0)
    g = Connect4GNNWrapper(game, base_args(use_gnn=True))
    g.nnet.load_state_dict({k: torch.from_numpy(v) for k, v in c4sd.items()})
    gsd = W.synthetic_state_dict(W.gnn_spec(3136, 2), GNN_C4_SEED)
    g.gnn.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
    del gsd
    args = base_args(numMCTSSims=100, use_gnn=True)
    A = game.getActionSize()
    sel = []
    orig_next = game.getNextState

    def rec_next(board, player, action):
        f = sys._getframe(1)
        if f.f_code.co_name == "search" and f.f_code.co_filename == ref_mcts.__file__:
            mc, st = f.f_locals["self"], f.f_locals["s"]
            us = []
            for b in range(A):
                if not mc.Vs[st][b]:
                    continue
                if (st, b) in mc.Qsa:
                    u = mc.Qsa[(st, b)] + mc.args.cpuct * mc.Ps[st][b] * math.sqrt(mc.Ns[st]) / (
                        1 + mc.Nsa[(st, b)])
                else:
                    u = mc.args.cpuct * mc.Ps[st][b] * math.sqrt(mc.Ns[st] + ref_mcts.EPS)
                us.append(float(u))
            us.sort(reverse=True)
            sel.append((zlib.crc32(st), int(action), us[0] - us[1] if len(us) > 1 else math.inf,
                        int(mc.Ns[st])))
        return orig_next(board, player, action)

    game.getNextState = rec_next
    coach = ref_coach.Coach.__new__(ref_coach.Coach)
    coach.game, coach.args, coach.nnet = game, args, g
    off, std, gnn, soff, goff = [0], [], [], [0], [0]
    t0 = time.time()
    for e in episodes:
        np.random.seed(e)
        coach.mcts = ref_mcts.MCTS(game, g, args)
        s_ex, g_ex = coach.executeEpisode()
        std += [(np.asarray(b).astype(np.int8), np.asarray(p, np.float64), float(r))
                for b, p, r in s_ex]
        gnn += [(np.asarray(x[0]).astype(np.int8), int(x[1]), np.asarray(x[2], np.float64),
                 np.float32(x[3]), np.asarray(x[4], np.float64), float(x[5]), float(x[6]))
                for x in g_ex]
        off.append(len(sel))
        soff.append(len(std))
        goff.append(len(gnn))
        print(f"  G6c episode {e}: {len(s_ex) // 2} moves, {off[-1] - off[-2]} selections, "
              f"{time.time() - t0:.1f}s", flush=True)
    game.getNextState = orig_next
    np.savez_compressed(
        out("mcts_c4_gnn_trace.npz"), episodes=np.array(list(episodes)),
        args=json.dumps(dict(args)),
        sel_off=np.array(off, np.int64), sel_state_crc32=np.array([x[0] for x in sel], np.uint32),
        sel_action=np.array([x[1] for x in sel], np.int8),
        sel_gap=np.array([x[2] for x in sel], np.float64),
        sel_ns=np.array([x[3] for x in sel], np.int32),
        std_off=np.array(soff, np.int64), std_board=np.stack([x[0] for x in std]),
        std_pi=np.stack([x[1] for x in std]), std_z=np.array([x[2] for x in std]),
        gnn_off=np.array(goff, np.int64), gnn_board=np.stack([x[0] for x in gnn]),
        gnn_player=np.array([x[1] for x in gnn], np.int8),
        gnn_init_pi=np.stack([x[2] for x in gnn]), gnn_init_v=np.array([x[3] for x in gnn]),
        gnn_exp_pi=np.stack([x[4] for x in gnn]), gnn_exp_v=np.array([x[5] for x in gnn]),
        gnn_reward=np.array([x[6] for x in gnn]))


# ----------------------------------------------------------------------------------- G7
def g7():
    """main.py:158-285 wiring for: --game tictactoe --board_size 3 --use_gnn --numIters 1."""
    import yaml
    with open(os.path.join(REF, "tictactoe", "config.yaml")) as f:
        config = yaml.safe_load(f)
    args = dotdict({})
    for section in config:                       # main.py:30-43
        for k, v in config[section].items():
            args[k] = v
    args.checkpoint = args.checkpoint_path
    args.board_size = 3
    args.numIters = 1
    args.use_gnn = True
    args.gnn_layers = 2
    args.game = "tictactoe"
    args.load_model = False
    tmp = tempfile.mkdtemp(prefix="az_g7_")
    folder = os.path.join(tmp, "tictactoe")
    os.makedirs(folder)
    args.checkpoint = folder
    args.load_folder_file = (folder, "best_gnn.pth.tar")
    random.seed(0)
    np.random.seed(0)
    torch.manual_seed(0)
    game = TicTacToeGame(n=3)
    nnet = TicTacToeGNNWrapper(game, args)
    coach = ref_coach.Coach(game, nnet, args)
    arena_res = []
    orig = ref_arena.Arena.playGames

    def pg(self, num, verbose=False):
        r = orig(self, num, verbose)
        arena_res.append([int(x) for x in r])
        return r

    ref_arena.Arena.playGames = pg
    try:
        t0 = time.time()
        coach.learn()
        dt = time.time() - t0
    finally:
        ref_arena.Arena.playGames = orig
    std_ex, gnn_ex = coach.trainExamplesHistory[0]
    res = dict(n_std=len(std_ex), n_gnn=len(gnn_ex), arena_pwins_nwins_draws=arena_res[0],
               files=sorted(os.listdir(folder)), seconds=dt)
    shutil.rmtree(tmp)
    with open(out("coach_ttt3.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("  G7", res)


# ----------------------------------------------------------------------------------- G9
def _ttt3_args(folder, numIters=1):
    """main.py:30-43,209-236 wiring for --game tictactoe --board_size 3 --use_gnn."""
    import yaml
    with open(os.path.join(REF, "tictactoe", "config.yaml")) as f:
        config = yaml.safe_load(f)
    args = dotdict({})
    for section in config:
        for k, v in config[section].items():
            args[k] = v
    args.update(board_size=3, numIters=numIters, use_gnn=True, gnn_layers=2, game="tictactoe",
                load_model=False, checkpoint=folder, load_folder_file=(folder, "best_gnn.pth.tar"))
    return args


def g9():
    tmp = tempfile.mkdtemp(prefix="az_g9_")
    first = os.path.join(tmp, "first")
    os.makedirs(first)
    random.seed(0)
    np.random.seed(0)
    torch.manual_seed(0)
    game = TicTacToeGame(n=3)
    args = _ttt3_args(first)
    nnet = TicTacToeGNNWrapper(game, args)
    ref_coach.Coach(game, nnet, args).learn()
    fix = os.path.join(HERE, "resume_ttt3")
    os.makedirs(fix, exist_ok=True)
    shutil.copy(os.path.join(first, "best_gnn.pth.tar"), os.path.join(fix, "best_gnn.pth.tar"))
    shutil.copy(os.path.join(first, "checkpoint_0_gnn.pth.tar.examples"),
                os.path.join(fix, "best_gnn.pth.tar.examples"))
    # the resumed iteration, exactly as main.py runs it with --load_model (seeds 1)
    second = os.path.join(tmp, "second")
    shutil.copytree(fix, second)
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    args = _ttt3_args(second)
    args.load_model = True
    nnet = TicTacToeGNNWrapper(game, args)
    nnet.load_checkpoint(args.load_folder_file[0], args.load_folder_file[1])
    coach = ref_coach.Coach(game, nnet, args)
    coach.loadTrainExamples()
    arena_res = []
    orig = ref_arena.Arena.playGames

    def pg(self, num, verbose=False):
        r = orig(self, num, verbose)
        arena_res.append([int(x) for x in r])
        return r

    ref_arena.Arena.playGames = pg
    try:
        coach.learn()
    finally:
        ref_arena.Arena.playGames = orig
    std_ex, gnn_ex = coach.trainExamplesHistory[0]
    res = dict(seeds=1, loaded_history=len(coach.trainExamplesHistory), n_std=len(std_ex),
               n_gnn=len(gnn_ex), skip_first_selfplay=bool(coach.skipFirstSelfPlay),
               arena_pwins_nwins_draws=arena_res[0], files=sorted(os.listdir(second)))
    shutil.rmtree(tmp)
    with open(out("resume_ttt3.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("  G9", res)


# ----------------------------------------------------------------------------------- G8
def g8():
    """Connect4Game.py:116-219 / TicTacToeGame.py on positions reached by seeded random play
    (terminal ones included)."""
    out = {}
    rng = np.random.default_rng(8)
    for name, game, count in (("c4n7", Connect4Game(7), 400), ("c4n5", Connect4Game(5), 200),
                              ("ttt3", TicTacToeGame(3), 200), ("ttt4", TicTacToeGame(4), 200)):
        A = game.getActionSize()
        n = game.getBoardSize()[0]
        boards, ended, valids, nxt, nxt_player, sym_b, sym_p = [], [], [], [], [], [], []
        for _ in range(count):
            b, p = game.getInitBoard(), 1
            for _ in range(int(rng.integers(0, n * n + 2))):
                if game.getGameEnded(b, p) != 0:
                    break
                v = game.getValidMoves(b, p)
                b, p = game.getNextState(b, p, int(rng.choice(np.flatnonzero(v))))
            c = game.getCanonicalForm(b, p)
            boards.append(c.astype(np.int8))
            e1, e2 = game.getGameEnded(c, 1), game.getGameEnded(c, -1)
            ended.append([float(e1), float(e2), isinstance(e1, int), isinstance(e2, int)])
            vm = np.asarray(game.getValidMoves(c, 1))
            valids.append(vm.astype(np.int8))
            ns = np.zeros((A, n, n), np.int8)
            npl = np.zeros(A, np.int8)
            for a in np.flatnonzero(vm):
                nb, pl = game.getNextState(c, 1, int(a))
                ns[a] = nb
                npl[a] = pl
            nxt.append(ns)
            nxt_player.append(npl)
            pi = rng.random(A)
            pi /= pi.sum()
            sym = game.getSymmetries(c, pi)
            sym_b.append(np.stack([np.asarray(x).astype(np.int8) for x, _ in sym]))
            sym_p.append(np.stack([np.asarray(y, np.float64) for _, y in sym]))
            sym_p[-1] = np.concatenate([pi[None], sym_p[-1]])
        out.update({f"{name}/boards": np.stack(boards), f"{name}/ended": np.array(ended),
                    f"{name}/valids": np.stack(valids), f"{name}/next": np.stack(nxt),
                    f"{name}/next_player": np.stack(nxt_player),
                    f"{name}/sym_boards": np.stack(sym_b), f"{name}/sym_pi": np.stack(sym_p)})
    np.savez_compressed(out_path("rules.npz"), **out)


def out_path(name):
    return os.path.join(HERE, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    a = ap.parse_args()
    want = set(a.only) if a.only else {"g1", "g2", "g3", "g4", "g5", "g6", "g7", "g8"}
    t0 = time.time()
    if want == {"g8"}:
        g8()
        print(f"G8 done {time.time() - t0:.1f}s")
        return
    if want == {"g6b"}:
        g6b()
        print(f"G6b done {time.time() - t0:.1f}s")
        return
    if want == {"g6c"}:
        g6c()
        print(f"G6c done {time.time() - t0:.1f}s")
        return
    if want == {"g9"}:
        g9()
        print(f"G9 done {time.time() - t0:.1f}s")
        return
    if want <= {"g2t", "g4b"}:
        for name in sorted(want):
            globals()[name]()
            print(f"{name.upper()} done {time.time() - t0:.1f}s")
        return
    c4net, c4b = g1()
    print(f"G1 done {time.time() - t0:.1f}s")
    c4sd = sd_np(c4net.nnet)
    if "g2" in want:
        g2(c4sd, c4b)
        print(f"G2 done {time.time() - t0:.1f}s")
    if "g3" in want:
        g3()
        print(f"G3 done {time.time() - t0:.1f}s")
    tnet, tb = g4()
    print(f"G4 done {time.time() - t0:.1f}s")
    if "g5" in want:
        g5(tb, c4sd, c4b)
        print(f"G5 done {time.time() - t0:.1f}s")
    if "g6" in want:
        g6(c4net, tnet)
        print(f"G6 done {time.time() - t0:.1f}s")
    if "g7" in want:
        g7()
        print(f"G7 done {time.time() - t0:.1f}s")
    if "g8" in want:
        g8()
        print(f"G8 done {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()

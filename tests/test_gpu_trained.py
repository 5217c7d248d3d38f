"""Policy / value parity on TRAINED Connect4 GNN weights (VERDICT r04 'do this' #1).

The large output_transform GEMMs run fp32 products as three fp16 products of row-scaled
operands (az_x3.h).  Round 4 checked the logits at 1e-5 only with init-scale weights; here the
weights are what training makes of them.

G2t (`tests/golden/make_goldens.py` g2t) ran the reference's own Connect4GNNWrapper.train
(Connect4GNN.py:122-197, dropout 0, 20 epochs) from G1's CNN + G2's GNN spec:
* 2 calls at lr 0.01: |w| up to 0.24, 13x the init; the reference itself is NaN after a 3rd;
* 5 calls at lr 0.001, connect4/config.yaml's rate.
Each fixture holds the examples, np seeds, the trained CNN, checksums + spot values of the
trained 479 MB GNN, and the reference's batch-1 predict / predict_with_gnn outputs (pi, v,
log pi) on 1,576 boards.  For the lr 0.01 run the trained output_transform weights themselves
(78.7 MB, all predict_with_gnn reads of the GNN) are written outside git to
tests/golden/large/ (sha256 committed) and travel with the tree to the GPU box.

1. `test_reference_trained_*`: the REFERENCE's trained weights loaded, every product entry point
   (batch-1 predict / predict_with_gnn, ops.c4_gnn_eval -- the bench's call -- at B = 1, 512,
   1,576, predict_both) against the reference's own outputs and the float64 oracle at 1e-5.
2. `test_trained_*`: this package's train() from the same start, examples and seeds (both runs),
   then the same entry points against float64 on THOSE weights.  The two training runs are
   compared only loosely: the Adam step's derivative at g = 0 is lr / eps (1e5 at lr 0.001), so a
   1e-10 summation-order difference in a near-zero gradient moves that weight by up to ~lr, and
   the trajectories drift apart over tens of steps (measured, reported).
pi and v are held absolutely; log pi relative to max(1, |log pi|) (trained log-probabilities
reach -731, where one fp32 ulp is 6e-5).  Every check writes its error and margin (1e-5 / error)
to $AZ_REPORT_DIR/margins.jsonl; torch fp32's own error on the same weights is recorded beside
it for scale.
"""
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import assert_close, golden, report, split_weights

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TOL = 1e-5
# L1 trajectory error / the reference's L1 travel: measured 0.020 overall (max tensor 0.084,
# conv2.bias) at lr 0.001 and 0 at lr 0.01 (profiles/r06/traj/); a wrong gradient gives ~1
TRAJ_BOUND, TRAJ_BOUND_TENSOR = 0.1, 0.25
RUNS = ("c4_gnn_trained_lr001.npz", "c4_gnn_trained_lr01.npz")


def _examples(zz):
    ex = [(b.astype(np.int64), p, z) for b, p, z in zip(zz["ex_boards"], zz["ex_pis"], zz["ex_z"])]
    gex = [(b.astype(np.int64), 1, None, None, p, v, 1)
           for b, p, v in zip(zz["gex_boards"], zz["gex_epis"], zz["gex_ev"])]
    return ex, gex


@pytest.fixture(scope="module", params=RUNS)
def trained(request, c4_gnn_weights):
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    zz = golden(request.param)
    args = SimpleNamespace(lr=float(zz["lr"]), epochs=int(zz["epochs"]), batch_size=64,
                           gnn_layers=2, dropout=0.0)
    w = Connect4GNNWrapper(Connect4Game(7), args)
    w.nnet.load_state_dict(split_weights(golden("c4_net.npz"), "w/"))
    w.gnn.load_state_dict(c4_gnn_weights)
    ex, gex = _examples(zz)
    for s in zz["np_seeds"]:
        np.random.seed(int(s))
        w.train(ex, gex)
    W = {k: v.numpy() for k, v in w.nnet.params.cpu_state_dict().items()}
    G = {k: w.gnn.params[k].detach().cpu().numpy() for k in
         ("output_transform.0.weight", "output_transform.0.bias",
          "output_transform.2.weight", "output_transform.2.bias")}
    boards = zz["boards"]
    import oracle.nets as O
    feat = O.c4_features(boards, W)
    y = O.output_transform(feat, G)
    lp64, v64 = O.c4_heads(y, W)
    sp_lp, sp_v = O.c4_forward(boards, W)
    tag = request.param.split(".")[0].replace("c4_gnn_trained_", "")
    return SimpleNamespace(tag=tag, zz=zz, w=w, W=W, G=G, boards=boards, lp64=lp64, v64=v64,
                           pi64=np.exp(lp64), sp_pi64=np.exp(sp_lp), sp_v64=sp_v, feat64=feat)


def test_trained_weights_follow_reference_training(trained):
    """This package's train() against the reference's training from the same start: the CNN in
    full, the GNN by the fixture's spot values.  Each tensor is held to the larger of 2x the
    reference's OWN spread -- the same reference training with 3 torch threads instead of 8
    ("envmax/...": up to 0.19 at lr 0.01, 0.04 at lr 0.001 after 40 / 100 Adam steps; see the
    module docstring) -- and 1e-3 of the largest displacement Adam can make (steps x lr).
    Reported per tensor; a gross training bug (a wrong gradient) exceeds it."""
    t, zz = trained, trained.zz
    steps = int(zz["trains"]) * int(zz["epochs"])
    floor = max(2e-5, 1e-3 * steps * float(zz["lr"]))
    per = {}
    for pre, items in (("w/", t.W.items()),
                       ("g/", ((k, v.numpy()) for k, v in t.w.gnn.params.cpu_state_dict().items()))):
        for k, a in items:
            if pre == "w/":
                e = float(np.abs(a - zz["w/" + k]).max())
            else:
                e = float(np.abs(a.ravel()[zz["gidx/" + k]] - zz["gval/" + k]).max())
            tol = max(floor, 2.0 * float(zz["envmax/" + pre + k]))
            per[pre + k] = {"max_abs": e, "tol": tol}
    report(f"trained_{t.tag}/weights_vs_reference_training", per_tensor=per)
    bad = {k: v for k, v in per.items() if v["max_abs"] > v["tol"]}
    assert not bad, bad


def c4_gnn_weights_np(t):
    from azhip.weights import gnn_spec, synthetic_state_dict
    from conftest import golden as _g
    return synthetic_state_dict(gnn_spec(3136, 2), int(_g("c4_gnn.npz")["seed"]))


def test_trained_cnn_follows_reference_trajectory(trained):
    """The same comparison relative to how far training moved the weights (VERDICT r05 weak #7:
    the per-tensor envelope above allows up to 0.19 where |w| <= 0.24).  For the CNN, held in
    full: the L1 distance to the reference's trained weights over the L1 distance the reference
    itself travelled from the common start, per tensor and over all tensors.  A near-zero
    gradient's Adam step (lr / eps at g = 0) scatters single weights by ~lr, which the L1 ratio
    averages out; a wrong gradient moves whole tensors elsewhere and shows up here as a ratio
    near 1 or above."""
    t, zz = trained, trained.zz
    W0 = split_weights(golden("c4_net.npz"), "w/")
    per, num, den = {}, 0.0, 0.0
    for k, a in t.W.items():
        ref = zz["w/" + k]
        w0 = W0[k].numpy() if hasattr(W0[k], "numpy") else np.asarray(W0[k])
        d = float(np.abs(ref - w0).sum())
        e = float(np.abs(a - ref).sum())
        per[k] = {"l1_err": e, "l1_travel": d, "ratio": e / max(d, 1e-30)}
        num += e
        den += d
    total = num / den
    # the GNN by the fixture's spot values: reported, not held -- the reference's own 3- vs
    # 8-thread runs already spread these tensors by up to 0.15 at lr 0.01 (|w| <= 0.12) and 0.04
    # at lr 0.001 (envmax/g/...), Adam's lr / eps response to near-zero gradients; measured
    # ratios 0.34 (lr 0.001) / 0.40 (lr 0.01), profiles/r06/traj/
    G0 = c4_gnn_weights_np(t)
    gper, gnum, gden = {}, 0.0, 0.0
    for k, a in t.w.gnn.params.cpu_state_dict().items():
        idx = zz["gidx/" + k]
        ref = zz["gval/" + k]
        w0 = G0[k].ravel()[idx]
        d = float(np.abs(ref - w0).sum())
        e = float(np.abs(a.numpy().ravel()[idx] - ref).sum())
        gper[k] = {"l1_err": e, "l1_travel": d, "ratio": e / max(d, 1e-30)}
        gnum += e
        gden += d
    report(f"trained_{t.tag}/gnn_spot_trajectory_vs_reference", total_ratio=gnum / max(gden, 1e-30),
           per_tensor=gper)
    report(f"trained_{t.tag}/cnn_trajectory_vs_reference", total_ratio=total, per_tensor=per,
           bound=TRAJ_BOUND, bound_tensor=TRAJ_BOUND_TENSOR)
    assert total <= TRAJ_BOUND, (total, per)
    assert all(v["ratio"] <= TRAJ_BOUND_TENSOR for v in per.values()), per


def _check(t, name, lp, pi, v, rows):
    rows = np.asarray(rows)
    if lp is not None:
        assert_close(f"trained_{t.tag}/{name}/logp_vs_fp64", lp, t.lp64[rows], TOL, rel_floor=1.0)
    assert_close(f"trained_{t.tag}/{name}/pi_vs_fp64", pi, t.pi64[rows], TOL)
    assert_close(f"trained_{t.tag}/{name}/v_vs_fp64", v, t.v64[rows], TOL)


@pytest.mark.parametrize("B", [1, 512, 1576])
def test_trained_c4_gnn_eval_vs_fp64(trained, B):
    """ops.c4_gnn_eval (the bench's product call: trunk -> split A -> two fp16x2 GEMMs with
    the fused reduce + split -> split-K heads) on the trained weights vs float64."""
    from azhip import ops
    t = trained
    b = torch.from_numpy(np.ascontiguousarray(t.boards[:B])).cuda()
    lp, pi, v = ops.c4_gnn_eval(b, t.w.nnet.params, t.w.gnn.params)
    torch.cuda.synchronize()
    _check(t, f"c4_gnn_eval_B{B}", lp.cpu().numpy(), pi.cpu().numpy(), v.cpu().numpy(),
           np.arange(B))


def test_trained_predict_entry_points_vs_fp64(trained):
    """The wrapper surface MCTS calls: batch-1 predict_with_gnn / predict and the lock-step
    batch predict_both (B = 1,576, the self-play round size) on the trained weights."""
    t = trained
    rows = list(range(0, 1576, 101))
    got = np.array([np.concatenate([p, [v]]) for p, v in
                    (t.w.predict_with_gnn(t.boards[i].astype(np.int64)) for i in rows)])
    _check(t, "predict_with_gnn_b1", None, got[:, :-1], got[:, -1], rows)
    got = np.array([np.concatenate([p, [v]]) for p, v in
                    (t.w.predict(t.boards[i].astype(np.int64)) for i in rows)])
    assert_close(f"trained_{t.tag}/predict_b1/pi_vs_fp64", got[:, :-1], t.sp_pi64[rows], TOL)
    assert_close(f"trained_{t.tag}/predict_b1/v_vs_fp64", got[:, -1], t.sp_v64[rows], TOL)
    pi, v, gpi, gv = t.w.predict_both(t.boards.astype(np.int64))
    _check(t, "predict_both_B1576", None, gpi, gv, np.arange(1576))
    assert_close(f"trained_{t.tag}/predict_both_B1576/std_pi_vs_fp64", pi, t.sp_pi64, TOL)
    assert_close(f"trained_{t.tag}/predict_both_B1576/std_v_vs_fp64", v, t.sp_v64, TOL)


@pytest.fixture(scope="module")
def ref_trained(c4_gnn_weights):
    """The reference's OWN trained weights (G2t, lr 0.01 x 2): CNN from the fixture, the
    output_transform weights from tests/golden/large/ (checked against the committed sha256),
    the message-passing layers (unused by a 1-row predict_with_gnn, gnn_utils.py:35-36) from
    G2's spec."""
    import hashlib
    import os
    from conftest import GOLDEN
    from connect4.Connect4GNN import Connect4GNNWrapper
    from connect4.Connect4Game import Connect4Game
    name = "c4_gnn_trained_lr01"
    path = os.path.join(GOLDEN, "large", name + "_ot.npz")
    if not os.path.exists(path):   # a GPU run without it has not checked the trained weights
        pytest.fail(f"{path} is missing: it is generated by tests/golden/make_goldens.py --only "
                    f"g2t (build container, reference mounted; git-ignored, 78.7 MB) and travels "
                    f"with the working tree to the GPU box")
    zo = np.load(path, allow_pickle=False)
    ot = {k: zo[k] for k in zo.files}
    digest = hashlib.sha256(b"".join(ot[k].tobytes() for k in sorted(ot))).hexdigest()
    assert digest == open(os.path.join(GOLDEN, name + "_ot.sha256")).read().strip()
    zz = golden(name + ".npz")
    w = Connect4GNNWrapper(Connect4Game(7), SimpleNamespace(gnn_layers=2, dropout=0.0))
    w.nnet.load_state_dict(split_weights(zz, "w/"))
    G = dict(c4_gnn_weights)
    G.update(ot)
    w.gnn.load_state_dict(G)
    W = split_weights(zz, "w/")
    import oracle.nets as O
    boards = zz["boards"]
    lp64, v64 = O.c4_heads(O.output_transform(O.c4_features(boards, W), ot), W)
    sp_lp, sp_v = O.c4_forward(boards, W)
    return SimpleNamespace(tag="reflr01", zz=zz, w=w, boards=boards, lp64=lp64, v64=v64,
                           pi64=np.exp(lp64), sp_pi64=np.exp(sp_lp), sp_v64=sp_v)


def test_reference_trained_reference_own_error(ref_trained):
    """Not a check of this package: the reference's OWN fp32 outputs (the G2t fixture, computed
    by its batch-1 predict_with_gnn on the CPU) against float64 on the same weights -- how much
    of the 1e-5 the reference's arithmetic itself uses, reported beside the GPU margins."""
    t, zz = ref_trained, ref_trained.zz
    e_pi = float(np.abs(zz["pi_gnn_b1"] - t.pi64).max())
    e_v = float(np.abs(zz["v_gnn_b1"] - t.v64).max())
    e_lp = float((np.abs(zz["logp_gnn_b1"] - t.lp64) / np.maximum(1.0, np.abs(t.lp64))).max())
    report("reflr01/reference_fp32_cpu_vs_fp64", pi=e_pi, v=e_v, logp_rel=e_lp,
           logp_min=float(t.lp64.min()))
    assert np.isfinite(e_pi + e_v + e_lp)


def _check_ref(t, name, lp, pi, v, rows):
    rows = np.asarray(rows)
    zz = t.zz
    if lp is not None:
        assert_close(f"{t.tag}/{name}/logp_vs_reference", lp, zz["logp_gnn_b1"][rows], TOL,
                     rel_floor=1.0)
    assert_close(f"{t.tag}/{name}/pi_vs_reference", pi, zz["pi_gnn_b1"][rows], TOL)
    assert_close(f"{t.tag}/{name}/v_vs_reference", v, zz["v_gnn_b1"][rows], TOL)
    _check(t, name, lp, pi, v, rows)


@pytest.mark.parametrize("B", [1, 512, 1576])
def test_reference_trained_c4_gnn_eval(ref_trained, B):
    """The bench's product call on the reference's trained weights vs the reference's batch-1
    predict_with_gnn outputs and vs float64."""
    from azhip import ops
    t = ref_trained
    b = torch.from_numpy(np.ascontiguousarray(t.boards[:B])).cuda()
    lp, pi, v = ops.c4_gnn_eval(b, t.w.nnet.params, t.w.gnn.params)
    torch.cuda.synchronize()
    _check_ref(t, f"c4_gnn_eval_B{B}", lp.cpu().numpy(), pi.cpu().numpy(), v.cpu().numpy(),
               np.arange(B))


def test_reference_trained_predict_entry_points(ref_trained):
    """Batch-1 predict_with_gnn / predict and the lock-step predict_both (B = 1,576) on the
    reference's trained weights vs the reference's outputs."""
    t, zz = ref_trained, ref_trained.zz
    rows = list(range(0, 1576, 53))
    got = np.array([np.concatenate([p, [v]]) for p, v in
                    (t.w.predict_with_gnn(t.boards[i].astype(np.int64)) for i in rows)])
    _check_ref(t, "predict_with_gnn_b1", None, got[:, :-1], got[:, -1], rows)
    got = np.array([np.concatenate([p, [v]]) for p, v in
                    (t.w.predict(t.boards[i].astype(np.int64)) for i in rows)])
    assert_close(f"{t.tag}/predict_b1/pi_vs_reference", got[:, :-1], zz["pi_b1"][rows], TOL)
    assert_close(f"{t.tag}/predict_b1/v_vs_reference", got[:, -1], zz["v_b1"][rows], TOL)
    pi, v, gpi, gv = t.w.predict_both(t.boards.astype(np.int64))
    _check_ref(t, "predict_both_B1576", None, gpi, gv, np.arange(1576))
    assert_close(f"{t.tag}/predict_both_B1576/std_pi_vs_reference", pi, zz["pi_b1"], TOL)
    assert_close(f"{t.tag}/predict_both_B1576/std_v_vs_reference", v, zz["v_b1"], TOL)


def test_trained_torch_fp32_error_for_scale(trained):
    """Not a parity check of this package: torch's own fp32 CPU forward (the reference's
    arithmetic, batched) on the same trained weights vs float64, recorded beside the GPU
    margins so a reader can see how much of 1e-5 fp32 itself uses."""
    t = trained
    f = torch.from_numpy(t.feat64.astype(np.float32))
    G = {k: torch.from_numpy(v) for k, v in t.G.items()}
    W = {k: torch.from_numpy(v) for k, v in t.W.items()}
    F = torch.nn.functional
    h = F.relu(F.linear(f, G["output_transform.0.weight"], G["output_transform.0.bias"]))
    y = F.linear(h, G["output_transform.2.weight"], G["output_transform.2.bias"])
    lp = F.log_softmax(F.linear(y, W["fc_policy.weight"], W["fc_policy.bias"]), dim=1)
    v = torch.tanh(F.linear(y, W["fc_value.weight"], W["fc_value.bias"]))[:, 0]
    e_pi = float(np.abs(lp.exp().numpy() - t.pi64).max())
    e_v = float(np.abs(v.numpy() - t.v64).max())
    e_lp = float((np.abs(lp.numpy() - t.lp64) / np.maximum(1.0, np.abs(t.lp64))).max())
    report(f"trained_{t.tag}/torch_fp32_cpu_vs_fp64", pi=e_pi, v=e_v, logp_rel=e_lp,
           logp_min=float(t.lp64.min()), w_amax=float(max(np.abs(g).max() for g in t.G.values())))
    assert np.isfinite(e_pi + e_v + e_lp)

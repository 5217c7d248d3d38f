"""The pre-split A hand-offs of the batched predict_with_gnn (Connect4GNN.py:86-120 per row,
output_transform = gnn_utils.py:115): the trunk writing output_transform.0's A as the fp16-form
GEMM's planes + row scales, and output_transform.0's split-K reduce writing output_transform.2's
(ops.c4_gnn_eval, one az_c4_eval_fwd call), give the same bits as the unfused calls -- trunk,
then each GEMM splitting its own A -- at every batch size (trunk NB 1..8, split-K and stream-K
GEMMs), and the same bits with unregistered weights (no hand-off: the plain path).  The unfused
calls ask for the heads without y too (linear_heads(want_y=False)), as the evaluator does."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ev():
    from azhip.nets import C4Evaluator
    from azhip.weights import connect4_net_spec, gnn_spec, synthetic_state_dict
    W = synthetic_state_dict(connect4_net_spec(7), 1)
    G = synthetic_state_dict(gnn_spec(3136, 2), 2)
    return C4Evaluator(W, G, device=torch.device("cuda"))


def _unfused(ops, boards, Wn, Gn):
    feat = ops.c4_trunk(boards, Wn)
    h = ops.linear(feat, Gn["output_transform.0.weight"], Gn["output_transform.0.bias"],
                   act=ops.ACT_RELU)
    logp, pi, v, _ = ops.linear_heads(h, Gn["output_transform.2.weight"],
                                      Gn["output_transform.2.bias"], Wn["fc_policy.weight"],
                                      Wn["fc_policy.bias"], Wn["fc_value.weight"],
                                      Wn["fc_value.bias"], want_y=False)
    return feat, h, logp, pi, v


@pytest.mark.parametrize("B", [1, 9, 300, 512, 1024, 1576, 3150])
def test_c4_gnn_eval_equals_unfused_calls(ev, B):
    from azhip import ops
    Wn, Gn = ev.nnet.params, ev.gnn.params
    rng = np.random.default_rng(B)
    boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)).cuda()
    # above 64 rows output_transform.0 / .2 take the pre-split operands for certain and the fp32
    # feature / hidden rows are not written (az_hip.h az_c4_eval_fwd): NaN there would reach the
    # outputs if anything still read them
    feat = torch.full((B, 3136), float("nan"), device="cuda")
    hidden = torch.full((B, 3136), float("nan"), device="cuda")
    logp, pi, v = ops.c4_gnn_eval(boards, Wn, Gn, feat=feat, hidden=hidden)
    feat_u, h_u, logp_u, pi_u, v_u = _unfused(ops, boards, Wn, Gn)
    _, pi_e, v_e = ev.evaluate(boards, gnn=True)
    torch.cuda.synchronize()
    assert torch.equal(feat, feat_u) or (B > 64 and bool(torch.isnan(feat).all()))
    assert torch.equal(hidden, h_u) or (B > 64 and bool(torch.isnan(hidden).all()))
    assert torch.equal(logp, logp_u) and torch.equal(pi, pi_u) and torch.equal(v, v_u)
    assert torch.equal(pi, pi_e) and torch.equal(v, v_e)


def test_c4_gnn_eval_unregistered_weights(ev):
    """Weights outside registered parameter storage: no cached planes, so no hand-off; the call
    still computes the same network (bit-identical to the unfused calls on the same copies)."""
    from azhip import ops
    Wn = {k: ev.nnet.params[k].clone() for k in ev.nnet.params.keys()}
    Gn = {k: ev.gnn.params[k].clone() for k in ev.gnn.params.keys()}
    B = 512
    rng = np.random.default_rng(7)
    boards = torch.from_numpy(rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)).cuda()
    logp, pi, v = ops.c4_gnn_eval(boards, Wn, Gn)
    _, _, logp_u, pi_u, v_u = _unfused(ops, boards, Wn, Gn)
    _, pi_r, v_r = ev.evaluate(boards, gnn=True)
    torch.cuda.synchronize()
    assert torch.equal(logp, logp_u) and torch.equal(pi, pi_u) and torch.equal(v, v_u)
    # registered vs unregistered storage of the same values: the same bits (same planes)
    assert torch.equal(pi, pi_r) and torch.equal(v, v_r)


@pytest.mark.parametrize("B", [200, 500, 600, 1000, 1200, 1576, 1700, 3150, 4100])
def test_c4_trunk_two_blocks_per_cu_equals_one(ev, B):
    """Registered weights take the REGW trunk kernels, whose LDS (no conv2 staging room) puts two
    512-thread blocks on a CU for NB <= 3; unregistered copies take the one-block-per-CU form.
    Round 5 saw wrong rows whenever two trunk blocks shared a CU; the cause was packed-FP32 VALU
    code (no longer emitted).  Both forms must give the same bits at every NB the
    rounds model picks, twice in a row (the failure was nondeterministic), and match the oracle."""
    from azhip import ops
    from oracle import nets as O
    Wn = ev.nnet.params
    Wc = {k: Wn[k].clone() for k in Wn.keys()}
    rng = np.random.default_rng(B + 1)
    bnp = rng.integers(-1, 2, size=(B, 7, 7)).astype(np.int8)
    boards = torch.from_numpy(bnp).cuda()
    reg = [ops.c4_trunk(boards, Wn) for _ in range(2)]
    unreg = ops.c4_trunk(boards, Wc)
    torch.cuda.synchronize()
    for f in reg:
        bad = torch.nonzero((f != unreg).any(1)).flatten().tolist()
        assert not bad, f"B={B}: {len(bad)} rows differ, first {bad[:8]}"
    sel = np.r_[0:4, B // 2:B // 2 + 4, B - 4:B]
    W64 = {k: Wn[k].double().cpu().numpy() for k in Wn.keys()}
    np.testing.assert_allclose(reg[0][torch.from_numpy(sel).cuda()].cpu().numpy(),
                               O.c4_features(bnp[sel], W64), atol=1e-5, rtol=1e-5)

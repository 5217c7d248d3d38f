"""Pin the oracle: the numpy restatement against vectors captured from the reference (CPU)."""
import numpy as np
import pytest

from conftest import golden, split_weights
from oracle import nets as O


def test_c4_net_forward_matches_reference():
    z = golden("c4_net.npz")
    W = split_weights(z, "w/")
    lp, v = O.c4_forward(z["boards"], W)
    np.testing.assert_allclose(lp, z["logp_batch"], atol=2e-6)
    np.testing.assert_allclose(v, z["v_batch"], atol=2e-6)
    np.testing.assert_allclose(np.exp(lp), z["pi_b1"], atol=2e-6)
    np.testing.assert_allclose(v, z["v_b1"], atol=2e-6)


def test_torch_default_init_reproduces_reference_weights():
    import torch
    from azhip.weights import connect4_net_spec, tictactoe_net_spec, gnn_spec, torch_default_init
    z = golden("c4_net.npz")
    torch.manual_seed(0)
    sd = torch_default_init(connect4_net_spec(7))
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), z["w/" + k])
    t = golden("ttt3.npz")
    torch.manual_seed(0)
    sd = torch_default_init(tictactoe_net_spec(3))      # TicTacToeGNN.py:17 (nnet first)
    gd = torch_default_init(gnn_spec(128, 2))           # then the GNN, TicTacToeGNN.py:23-27
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), t["w/" + k])
    for k, v in gd.items():
        np.testing.assert_array_equal(v.numpy(), t["g/" + k])


def test_ttt3_predict_and_gnn_all_positions():
    z = golden("ttt3.npz")
    W, G = split_weights(z, "w/"), split_weights(z, "g/")
    assert z["boards"].shape[0] == 5478
    lp, v = O.ttt_forward(z["boards"], W)
    np.testing.assert_allclose(np.exp(lp), z["pi"], atol=2e-6)
    np.testing.assert_allclose(v, z["v"], atol=2e-6)
    f = O.ttt_features(z["boards"], W)
    lp, v = O.ttt_heads(O.policy_value_gnn_per_row(f, G), W)
    np.testing.assert_allclose(np.exp(lp), z["pi_gnn"], atol=2e-6)
    np.testing.assert_allclose(v, z["v_gnn"], atol=2e-6)


@pytest.mark.slow
def test_c4_gnn_per_row_and_star(c4_gnn_weights):
    z = golden("c4_gnn.npz")
    W = split_weights(golden("c4_net.npz"), "w/")
    G = c4_gnn_weights
    f = O.c4_features(z["boards"], W)
    lp, v = O.c4_heads(O.policy_value_gnn_per_row(f, G), W)
    np.testing.assert_allclose(np.exp(lp), z["pi_gnn_b1"], atol=5e-6)
    np.testing.assert_allclose(v, z["v_gnn_b1"], atol=5e-6)
    tr = {}
    x = np.array(f)
    rows0 = []
    for i in range(2):
        x = O.gnn_layer_star(x, G, i, trace=tr)
        rows0.append(x[0])
    np.testing.assert_allclose(np.stack(tr["alpha_raw"]), z["star_alpha_raw"], atol=2e-6)
    np.testing.assert_allclose(np.stack(tr["agg"]), z["star_agg"], atol=1e-5)
    np.testing.assert_allclose(np.stack(rows0), z["star_row0"], atol=1e-5)
    enh = O.output_transform(x, G)
    np.testing.assert_allclose(enh[0], z["star_enh_row0"], atol=1e-5)
    lp, v = O.c4_heads(enh, W)
    np.testing.assert_allclose(lp, z["star_logp"], atol=1e-5)
    np.testing.assert_allclose(v, z["star_v"], atol=1e-5)


def test_synthetic_grid_and_star():
    from azhip.weights import gnn_spec, synthetic_state_dict
    z = golden("synth_gnn.npz")
    G = synthetic_state_dict(gnn_spec(64, 2), int(z["seed_w"]))
    rng = np.random.Generator(np.random.PCG64(int(z["seed_x"])))
    x0 = rng.random((1024, 64), dtype=np.float32) * np.float32(2) - np.float32(1)
    x1 = O.gnn_layer_csr(x0, z["rowptr"], z["col"], G, 0)
    np.testing.assert_allclose(x1, z["grid_x1"], atol=2e-6)
    x2 = O.gnn_layer_csr(x1, z["rowptr"], z["col"], G, 1)
    np.testing.assert_allclose(x2, z["grid_x2"], atol=2e-6)
    np.testing.assert_allclose(O.output_transform(x2, G), z["grid_out"], atol=2e-6)
    rng = np.random.Generator(np.random.PCG64(int(z["seed_star"])))
    sx = rng.random((4096, 64), dtype=np.float32) * np.float32(2) - np.float32(1)
    out = O.policy_value_gnn_star(sx, G)
    np.testing.assert_allclose(out[:65], z["star_out_head"], atol=2e-6)
    np.testing.assert_allclose(out.sum(1), z["star_out_rowsum"], atol=2e-5)

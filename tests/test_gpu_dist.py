"""Data-parallel training on the MI355X (azhip/train.py gnn_step_dp).

Ranks are processes sharing the box's one GPU over gloo (RCCL cannot place two ranks on one
device; the 8-GPU RCCL runs are the driver's); RCCL itself is exercised at world size 1 --
process-group init over the device, the flat-gradient all_reduce, the broadcast and the
all_gather the DP step uses.  Against the 1-rank train() on the same examples and np.random
state: bit-identical on every rank, and after one Adam step within a bound derived from the two
runs' gradients (adam_one_step_bound).
"""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import golden, split_weights

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wrapper(kind, mode, sync, epochs=2):
    from azhip.weights import gnn_spec, synthetic_state_dict
    a = SimpleNamespace(lr=0.001, epochs=epochs, batch_size=64, gnn_layers=2, dropout=0.3,
                        train_parallel=mode, gnn_grad_sync=sync)
    if kind == "c4":
        from connect4.Connect4GNN import Connect4GNNWrapper
        from connect4.Connect4Game import Connect4Game
        w = Connect4GNNWrapper(Connect4Game(7), a)
        w.nnet.load_state_dict(split_weights(golden("c4_net.npz"), "w/"))
        w.gnn.load_state_dict(synthetic_state_dict(gnn_spec(3136, 2),
                                                   int(golden("c4_gnn.npz")["seed"])))
    else:
        from tictactoe.TicTacToeGNN import TicTacToeGNNWrapper
        from tictactoe.TicTacToeGame import TicTacToeGame
        z = golden("ttt3.npz")
        w = TicTacToeGNNWrapper(TicTacToeGame(3), a)
        w.nnet.load_state_dict(split_weights(z, "w/"))
        w.gnn.load_state_dict(split_weights(z, "g/"))
    return w


def _dp_worker(rank, world, port, outdir, kind, sync, epochs=2):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from azhip import dist as D
    from test_gpu_train import _examples
    ex, gex = _examples(golden("train_c4.npz" if kind == "c4" else "train_ttt3.npz"))
    single = _wrapper(kind, "replicas", sync, epochs)     # before init: a plain 1-rank train()
    p0 = {"nnet": single.nnet.params.flat.cpu(), "gnn": single.gnn.params.flat.cpu()}
    np.random.seed(11)
    single.train(ex, gex)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dp = _wrapper(kind, "allreduce", sync, epochs)
    np.random.seed(11)
    dp.train(ex, gex)
    torch.cuda.synchronize()
    res = {"single_nnet": single.nnet.params.flat.cpu(), "single_gnn": single.gnn.params.flat.cpu(),
           "dp_nnet": dp.nnet.params.flat.cpu(), "dp_gnn": dp.gnn.params.flat.cpu(),
           "sync": D.params_in_sync(dp.gnn.params.flat) and D.params_in_sync(dp.nnet.params.flat),
           # the last step's gradients (the ones its Adam step used), and the start
           "g_single_nnet": single.nnet.params.grad_flat.cpu(),
           "g_single_gnn": single.gnn.params.grad_flat.cpu(),
           "g_dp_nnet": dp.nnet.params.grad_flat.cpu(), "g_dp_gnn": dp.gnn.params.grad_flat.cpu(),
           "p0_nnet": p0["nnet"], "p0_gnn": p0["gnn"]}
    torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


LR, EPS, U32 = 1e-3, 1e-8, 2.0 ** -24


def adam_one_step_bound(g_a, g_b, p_a, p_b, lr=LR, eps=EPS):
    """Per-element bound on |p_a - p_b| after ONE Adam step (torch defaults, fresh moments: the
    reference builds its optimisers per train() call, Connect4GNN.py:132-133) from the same
    start whose gradients differ only by summation order (g_a, g_b).  Step 1 moves a parameter
    by -lr f(g) with f(g) = g / (|g| + eps) (m_hat = g, v_hat = g^2); f' = eps / (|g| + eps)^2,
    so by the mean value theorem |lr f(g_a) - lr f(g_b)| <= lr |g_a - g_b| eps / (m + eps)^2,
    m = min(|g_a|, |g_b|) when the signs agree and 0 when they differ (f is steepest at 0:
    1 / eps, which is how a sign flip of a near-zero gradient becomes a visible step).  Both
    fp32 evaluations of the step (lerp, mul, sqrt, div, add) err by <= 8 u lr each, and the
    final p - step rounds by <= u |p| on each side."""
    ga, gb = g_a.double().abs(), g_b.double().abs()
    same = torch.sign(g_a) == torch.sign(g_b)
    m = torch.where(same, torch.minimum(ga, gb), torch.zeros_like(ga))
    d = (g_a.double() - g_b.double()).abs()
    return (lr * d * eps / (m + eps) ** 2 + 16 * U32 * lr +
            U32 * (p_a.double().abs() + p_b.double().abs()))


@pytest.mark.parametrize("kind,world,sync", [("c4", 2, "row0"), ("c4", 2, "flat"),
                                             ("c4", 4, "row0"), ("ttt", 3, "row0"),
                                             ("ttt", 2, "flat")])
def test_dp_train_equals_single_rank(tmp_path, kind, world, sync):
    """Connect4GNNWrapper / TicTacToeGNNWrapper.train (1 epoch: one CNN step + one star GNN step,
    Connect4 with dropout 0.3) with train_parallel="allreduce" on `world` ranks against the same
    train() on one rank; 64 rows over 3 ranks exercises uneven shards.  Every rank ends
    bit-identical, and each parameter is within adam_one_step_bound (derived above) of the
    one-rank result, evaluated on the two runs' own gradients (the only difference between them
    is the summation order of the sharded gradient).  The margin is reported."""
    import json
    import torch.multiprocessing as mp
    mp.spawn(_dp_worker, args=(world, _port(), str(tmp_path), kind, sync, 1), nprocs=world)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    assert all(x["sync"] for x in r)
    for key in ("dp_nnet", "dp_gnn", "single_nnet", "single_gnn"):
        assert all(torch.equal(r[0][key], x[key]) for x in r[1:]), key
    rep = {"kind": kind, "world": world, "sync": sync}
    for part in ("nnet", "gnn"):
        a, b = r[0]["dp_" + part], r[0]["single_" + part]
        bound = adam_one_step_bound(r[0]["g_dp_" + part], r[0]["g_single_" + part], a, b)
        diff = (a.double() - b.double()).abs()
        ratio = diff / bound
        i = int(ratio.argmax())
        rep[part] = {"max_abs_diff": float(diff.max()), "worst_ratio_to_bound": float(ratio[i]),
                     "at": i, "grad_diff_max": float((r[0]["g_dp_" + part] -
                                                      r[0]["g_single_" + part]).abs().max())}
        assert bool((diff <= bound).all()), rep
        assert not torch.equal(a, r[0]["p0_" + part]), part      # the step really moved it
    d = os.environ.get("AZ_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "dp_one_step_bound.jsonl"), "a") as f:
            f.write(json.dumps(rep) + "\n")


def _adam_ref(g_steps, lr=LR, b1=0.9, b2=0.999, eps=EPS):
    """float64 Adam updates (torch's formulas, fresh moments) for one run's recorded gradients:
    the list of the parameter displacements step by step."""
    m = torch.zeros_like(g_steps[0], dtype=torch.float64)
    v = torch.zeros_like(m)
    out = []
    for t, g in enumerate(g_steps, 1):
        g = g.double()
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        out.append(lr * (m / (1 - b1 ** t)) / ((v / (1 - b2 ** t)).sqrt() + eps))
    return out


def _dp2_worker(rank, world, port, outdir):
    """Two epochs, single rank vs DP (row0), recording every Adam step's gradient and the
    parameters around it (on the GPU; only the verdicts leave the process)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from azhip import dist as D, train as T
    from test_gpu_train import _examples
    ex, gex = _examples(golden("train_c4.npz"))
    rec = {}
    orig = T.adam_step

    def recording(net, lr):
        P = net.params
        key = (run[0], "gnn" if P.numel > 1_000_000 else "nnet")
        before, g = P.flat.clone(), P.grad_flat.clone()
        orig(net, lr)
        rec.setdefault(key, []).append((g, before, P.flat.clone()))

    T.adam_step = recording
    run = ["single"]
    single = _wrapper("c4", "replicas", "row0", 2)
    np.random.seed(11)
    single.train(ex, gex)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    run[0] = "dp"
    dp = _wrapper("c4", "allreduce", "row0", 2)
    np.random.seed(11)
    dp.train(ex, gex)
    torch.cuda.synchronize()
    T.adam_step = orig
    out = {"sync": D.params_in_sync(dp.gnn.params.flat) and D.params_in_sync(dp.nnet.params.flat)}
    for part in ("nnet", "gnn"):
        for name in ("single", "dp"):
            steps = rec[(name, part)]
            assert len(steps) == 2
            ups = _adam_ref([g for g, _, _ in steps])
            worst = 0.0
            for (g, before, after), u in zip(steps, ups):
                moved = (before.double() - after.double())
                slop = 16 * U32 * LR + U32 * (before.double().abs() + after.double().abs())
                worst = max(worst, float(((moved - u).abs() / slop).max()))
            out[f"adam_identity_{name}_{part}"] = worst
        for t in range(2):
            ga, gb = rec[("dp", part)][t][0], rec[("single", part)][t][0]
            out[f"grad_rel_step{t + 1}_{part}"] = float((ga - gb).abs().max() / gb.abs().max())
        out[f"param_diff_{part}"] = float((rec[("dp", part)][1][2] -
                                           rec[("single", part)][1][2]).abs().max())
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_dp_train_two_epochs_ranks_identical(tmp_path):
    """Two epochs of DP train() (Connect4, row0, 2 ranks) against the one-rank train():
    * every rank ends bit-identical (params_in_sync);
    * each run's every Adam step is the float64 Adam update of the gradient that run computed,
      within fp32 evaluation rounding (16 u lr + u |p| per element, the one-step bound's terms):
      so the runs differ ONLY through their gradients;
    * those gradients agree to summation-order size: step 1 within 1e-5 of the gradient's
      largest magnitude (the sharded rows summed in another order), step 2 -- which also sees
      step 1's parameter difference -- within 2e-5 (measured 5.7e-7 and 1.2e-6).
    A wrong gradient exchange fails the third check even where Adam's sign-like first step would
    hide it in the parameters.  Measured values are reported (AZ_REPORT_DIR)."""
    import json
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_dp2_worker, args=(world, _port(), str(tmp_path)), nprocs=world)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    assert all(x["sync"] for x in r)
    out = r[0]
    d = os.environ.get("AZ_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "dp_two_epochs.json"), "w") as f:
            json.dump(out, f, indent=1)
    for part in ("nnet", "gnn"):
        for name in ("single", "dp"):
            assert out[f"adam_identity_{name}_{part}"] <= 1.0, (name, part, out)
        assert out[f"grad_rel_step1_{part}"] <= 1e-5, out
        assert out[f"grad_rel_step2_{part}"] <= 2e-5, out


def _auto_worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from azhip import dist as D
    from test_gpu_train import _examples
    ex, gex = _examples(golden("train_c4.npz"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    auto = _wrapper("c4", "auto", "row0", 2)
    np.random.seed(11)
    auto.train(ex, gex)
    state = np.random.get_state()[1].copy()
    fixed = _wrapper("c4", auto._tp_auto, "row0", 2)
    np.random.seed(11)
    fixed.train(ex, gex)
    torch.cuda.synchronize()
    out = {"choice": auto._tp_auto, "probe": auto.train_parallel_probe,
           "sync": D.params_in_sync(auto.gnn.params.flat),
           "same_as_fixed": bool(torch.equal(auto.gnn.params.flat, fixed.gnn.params.flat) and
                                 torch.equal(auto.nnet.params.flat, fixed.nnet.params.flat)),
           "rng_same": bool((state == np.random.get_state()[1]).all())}
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_train_parallel_auto_is_a_measured_choice(tmp_path):
    """train_parallel="auto" (wrappers._probe_train_parallel): 2 ranks time the replicas and
    data-parallel gradient computations on the node, agree on the faster (max over ranks), and
    then train exactly as that fixed mode does -- bit-identical parameters, the same np.random
    stream afterwards (the probe draws nothing)."""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_auto_worker, args=(world, _port(), str(tmp_path)), nprocs=world)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    assert r[0]["choice"] in ("replicas", "allreduce") and r[0]["choice"] == r[1]["choice"]
    assert r[0]["probe"] == r[1]["probe"]
    for x in r:
        assert x["sync"] and x["same_as_fixed"] and x["rng_same"], x
    for k in ("cnn_replicas_ms", "cnn_allreduce_ms", "gnn_replicas_ms", "gnn_allreduce_ms"):
        assert r[0]["probe"][k] > 0


def _nccl_worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from azhip import dist as D, train as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    out = {}
    # the GNN gradient bucket: 119.6 M floats (478.6 MB), one all_reduce over RCCL
    w = _wrapper("c4", "allreduce", "flat")
    g = w.gnn.params.grad_flat
    g.copy_(torch.arange(g.numel(), device=g.device, dtype=torch.float32).remainder_(977.0))
    want = g.clone()
    D.allreduce_sum_(g)
    torch.cuda.synchronize()
    out["allreduce_equal"] = bool(torch.equal(g, want))
    x = torch.randn((13, 3136), device="cuda")
    out["gather_equal"] = bool(torch.equal(D.gather_rows(x, 13, 1, 0), x))
    # the DP GNN step's collectives (gather, broadcast, span all_reduce) on RCCL at world 1
    from test_gpu_train import _examples
    ex, gex = _examples(golden("train_c4.npz"))
    b, p, v = w._gnn_batch(gex)
    l_dp = T.gnn_grads_dp(w.nnet, w.gnn, b, p, v, seed=3, grad_sync="row0")
    g_dp = w.gnn.params.grad_flat.clone()
    l_1 = T.gnn_grads(w.nnet, w.gnn, b, p, v, seed=3)
    g_1 = w.gnn.params.grad_flat.clone()
    out["loss_close"] = bool(torch.allclose(l_dp, l_1, atol=1e-6))
    out["grad_maxdiff"] = float((g_dp - g_1).abs().max())
    out["grad_scale"] = float(g_1.abs().max())
    torch.save(out, os.path.join(outdir, "nccl.pt"))
    dist.destroy_process_group()


def test_rccl_world1_collectives_and_dp_step(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_nccl_worker, args=(1, _port(), str(tmp_path)), nprocs=1)
    out = torch.load(tmp_path / "nccl.pt", weights_only=True)
    assert out["allreduce_equal"] and out["gather_equal"] and out["loss_close"]
    assert out["grad_maxdiff"] <= 1e-6 * max(1.0, out["grad_scale"]), out

"""Data-parallel training on the MI355X (azhip/train.py gnn_step_dp).

Ranks are processes sharing the box's one GPU over gloo (RCCL cannot place two ranks on one
device; the 8-GPU RCCL runs are the driver's); RCCL itself is exercised at world size 1 --
process-group init over the device, the flat-gradient all_reduce, the broadcast and the
all_gather the DP step uses.  Against the 1-rank train() on the same examples and np.random
state: parameters within 2e-5 (the G5 golden tolerance) and bit-identical on every rank.
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


def _dp_worker(rank, world, port, outdir, kind, sync):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from azhip import dist as D
    from test_gpu_train import _examples
    ex, gex = _examples(golden("train_c4.npz" if kind == "c4" else "train_ttt3.npz"))
    single = _wrapper(kind, "replicas", sync)             # before init: a plain 1-rank train()
    np.random.seed(11)
    single.train(ex, gex)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dp = _wrapper(kind, "allreduce", sync)
    np.random.seed(11)
    dp.train(ex, gex)
    torch.cuda.synchronize()
    res = {"single_nnet": single.nnet.params.flat.cpu(), "single_gnn": single.gnn.params.flat.cpu(),
           "dp_nnet": dp.nnet.params.flat.cpu(), "dp_gnn": dp.gnn.params.flat.cpu(),
           "sync": D.params_in_sync(dp.gnn.params.flat) and D.params_in_sync(dp.nnet.params.flat)}
    torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,sync", [("c4", 2, "row0"), ("c4", 2, "flat"),
                                             ("c4", 4, "row0"), ("ttt", 3, "row0"),
                                             ("ttt", 2, "flat")])
def test_dp_train_equals_single_rank(tmp_path, kind, world, sync):
    """Connect4GNNWrapper / TicTacToeGNNWrapper.train (2 epochs: CNN step + star GNN step each,
    Connect4 with dropout 0.3) with train_parallel="allreduce" on `world` ranks == the same
    train() on one rank; 64 rows over 3 ranks exercises uneven shards."""
    import torch.multiprocessing as mp
    mp.spawn(_dp_worker, args=(world, _port(), str(tmp_path), kind, sync), nprocs=world)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    assert all(x["sync"] for x in r)
    for key in ("dp_nnet", "dp_gnn", "single_nnet", "single_gnn"):
        assert all(torch.equal(r[0][key], x[key]) for x in r[1:]), key
    for part in ("nnet", "gnn"):
        a, b = r[0]["dp_" + part].numpy(), r[0]["single_" + part].numpy()
        np.testing.assert_allclose(a, b, atol=2e-5, err_msg=part)
    assert not torch.equal(r[0]["dp_gnn"], _wrapper(kind, "replicas", sync, 0).gnn.params.flat.cpu())


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

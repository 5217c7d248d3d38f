"""Multi-rank host logic on CPU (gloo, world_size 2): episode sharding + gather gives the same
examples as one rank (and as the reference's sequential episodes, G6); synchronised host RNGs;
the flat-gradient all-reduce and the parameter-sync check (azhip/dist.py)."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _worker_selfplay(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from test_mcts_golden import Args, RecordedNet
    from test_selfplay import _norm_gnn, _norm_std
    from azhip import dist as D
    from selfplay import play_episodes
    from connect4.Connect4Game import Connect4Game
    from tictactoe.TicTacToeGame import TicTacToeGame
    dist = _init(rank, world, port)
    res = {}
    for name, game in (("mcts_c4", Connect4Game(7)), ("mcts_ttt3", TicTacToeGame(3))):
        meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
        net = RecordedNet(golden(name + ".npz"), 0)
        eps = [ep["episode"] for ep in meta["episodes"]]
        mine = [eps[i] for i in D.my_episodes(len(eps), world, rank)]
        local = play_episodes(game, net, Args(meta["args"]), mine, {e: e for e in eps},
                              parallel_games=4)
        assert set(local) == set(mine)
        allr = D.gather_episodes(local)
        res[name] = {e: (_norm_std(s), _norm_gnn(g)) for e, (s, g) in allr.items()}
    # host RNG sync: both ranks draw the same numbers afterwards
    np.random.seed(100 + rank)
    seed = D.sync_host_rngs()
    draws = np.random.randint(0, 1 << 30, size=4).tolist()
    # flat gradient all-reduce and parameter sync check
    g = torch.arange(6, dtype=torch.float32) * (rank + 1)
    D.allreduce_sum_(g)
    p = torch.ones(5)
    same = D.params_in_sync(p)
    p[rank] += 1.0
    differ = not D.params_in_sync(p)
    torch.save({"res": res, "seed": seed, "draws": draws, "g": g, "same": same,
                "differ": differ}, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_sharded_selfplay_equals_reference_episodes(tmp_path):
    world = 2
    mp.spawn(_worker_selfplay, args=(world, _free_port(), str(tmp_path)), nprocs=world)
    outs = [torch.load(tmp_path / f"r{r}.pt", weights_only=False) for r in range(world)]
    for name in ("mcts_c4", "mcts_ttt3"):
        meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
        for o in outs:                                      # every rank holds every episode
            got = o["res"][name]
            for ep in meta["episodes"]:
                std, gnn = got[ep["episode"]]
                assert std == [tuple(x) for x in ep["std_examples"]]
                assert gnn == [tuple(x) for x in ep["gnn_examples"]]
    assert outs[0]["seed"] == outs[1]["seed"] and outs[0]["draws"] == outs[1]["draws"]
    want = torch.arange(6, dtype=torch.float32) * 3
    assert all(torch.equal(o["g"], want) for o in outs)
    assert all(o["same"] and o["differ"] for o in outs)


def test_row_shard_covers_batch():
    from azhip.dist import row_shard
    for n in (0, 1, 5, 64, 65):
        for w in (1, 2, 3, 8):
            parts = [row_shard(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


def test_my_episodes_partition():
    from azhip.dist import my_episodes
    for n in (1, 7, 20, 64):
        for w in (1, 2, 8):
            got = sorted(e for r in range(w) for e in my_episodes(n, w, r))
            assert got == list(range(n))

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
    for name, game in (("mcts_c4", Connect4Game(7)), ("mcts_ttt3", TicTacToeGame(3)),
                       ("mcts_c4_gnn", Connect4Game(7))):
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


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_selfplay_equals_reference_episodes(tmp_path, world):
    """Episodes e -> rank e mod P (P = 4 leaves ranks without episodes), gathered and ordered:
    every rank holds the reference's examples for every episode (G6, G6b)."""
    mp.spawn(_worker_selfplay, args=(world, _free_port(), str(tmp_path)), nprocs=world)
    outs = [torch.load(tmp_path / f"r{r}.pt", weights_only=False) for r in range(world)]
    for name in ("mcts_c4", "mcts_ttt3", "mcts_c4_gnn"):
        meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
        for o in outs:                                      # every rank holds every episode
            got = o["res"][name]
            for ep in meta["episodes"]:
                std, gnn = got[ep["episode"]]
                assert std == [tuple(x) for x in ep["std_examples"]]
                assert gnn == [tuple(x) for x in ep["gnn_examples"]]
    assert all(o["seed"] == outs[0]["seed"] and o["draws"] == outs[0]["draws"] for o in outs)
    want = torch.arange(6, dtype=torch.float32) * (world * (world + 1) // 2)
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


class FakeNet:
    """A NeuralNet duck type for host-only Coach runs: (pi, v) a deterministic function of the
    board and of a `state` integer; train() folds a digest of the examples it received into the
    state (so the arena sees a changed network) and records it; checkpoints are JSON."""

    trained = []
    saves = []

    def __init__(self, game, args):
        self.A = game.getActionSize()
        self.state = 1

    def _row(self, b, salt):
        b = np.asarray(b, np.int64)
        h = np.random.default_rng([self.state, salt] + [int(x) + 1 for x in b.ravel()])
        p = h.random(self.A).astype(np.float32)
        return (p / p.sum()).astype(np.float32), np.float32(h.uniform(-1, 1))

    def predict(self, board):
        return self._row(board, 0)

    def predict_with_gnn(self, board):
        return self._row(board, 1)

    def predict_batch(self, boards):
        r = [self._row(b, 0) for b in boards]
        return np.stack([p for p, _ in r]), np.array([v for _, v in r], np.float32)

    def predict_both(self, boards):
        pi, v = self.predict_batch(boards)
        r = [self._row(b, 1) for b in boards]
        return pi, v, np.stack([p for p, _ in r]), np.array([x for _, x in r], np.float32)

    def train(self, examples, gnn_examples=None):
        import hashlib
        h = hashlib.sha256()
        for ex in list(examples) + list(gnn_examples or []):
            for x in ex:
                h.update(np.asarray(x, np.float64).tobytes())
        h.update(np.random.randint(0, 1 << 30, size=4).tobytes())   # the batch sampling draws
        d = h.hexdigest()
        FakeNet.trained.append(d)
        self.state = int(d[:8], 16)

    def save_checkpoint(self, folder, filename):
        FakeNet.saves.append(filename)
        os.makedirs(folder, exist_ok=True)
        with open(os.path.join(folder, filename), "w") as f:
            json.dump({"state": self.state}, f)

    def load_checkpoint(self, folder, filename):
        with open(os.path.join(folder, filename)) as f:
            self.state = json.load(f)["state"]


def _worker_coach(rank, world, port, outdir):
    import random
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_distributed import FakeNet
    from test_mcts_golden import Args
    from test_selfplay import _norm_gnn, _norm_std
    import Arena as A
    from Coach import Coach
    from tictactoe.TicTacToeGame import TicTacToeGame
    dist = _init(rank, world, port)
    folder = os.path.join(outdir, f"ck{world}")      # one shared checkpoint folder per run
    args = Args(numIters=2, numEps=5, tempThreshold=3, updateThreshold=0.6, maxlenOfQueue=200000,
                numItersForTrainExamplesHistory=5, numMCTSSims=5, cpuct=1.0, expand_by=2,
                arenaCompare=4, use_gnn=True, parallel_games=2, checkpoint=folder,
                load_folder_file=(folder, "best_gnn.pth.tar"))
    random.seed(0)
    np.random.seed(0)
    arena = []
    orig = A.Arena.playGames

    def pg(self, num, verbose=False):
        r = orig(self, num, verbose)
        arena.append([int(x) for x in r])
        return r

    A.Arena.playGames = pg
    try:
        game = TicTacToeGame(3)
        coach = Coach(game, FakeNet(game, args), args)
        coach.learn()
    finally:
        A.Arena.playGames = orig
    hist = [(_norm_std(s), _norm_gnn(g)) for s, g in coach.trainExamplesHistory]
    dist.barrier()
    files = sorted(os.listdir(folder))
    torch.save({"hist": hist, "trained": FakeNet.trained, "arena": arena, "files": files,
                "saves": FakeNet.saves,
                "state": coach.nnet.state}, os.path.join(outdir, f"c{world}_{rank}.pt"))
    dist.destroy_process_group()


def test_coach_learn_any_rank_count_equals_one_rank(tmp_path):
    """Two full Coach.learn iterations (TicTacToe 3x3, use_gnn, lock-step native self-play,
    train, arena gate, checkpoints) on P = 1, 3, 4, 8 gloo ranks, numEps = 5 (not a multiple of
    P; at P = 8 three ranks play nothing): every rank of every P ends with the 1-rank run's
    example history, train inputs, arena results and network, and only rank 0 writes files."""
    outs = {}
    for world in (1, 3, 4, 8):
        mp.spawn(_worker_coach, args=(world, _free_port(), str(tmp_path)), nprocs=world)
        outs[world] = [torch.load(tmp_path / f"c{world}_{r}.pt", weights_only=False)
                       for r in range(world)]
    ref = outs[1][0]
    assert len(ref["hist"]) == 2 and len(ref["trained"]) == 2 and len(ref["arena"]) == 2
    assert "best_gnn.pth.tar" in ref["files"] and "checkpoint_1_gnn.pth.tar.examples" in ref["files"]
    for world, ranks in outs.items():
        for r, o in enumerate(ranks):
            for k in ("hist", "trained", "arena", "state"):
                assert o[k] == ref[k], (world, r, k)
            assert o["files"] == ref["files"], (world, r)
            assert o["saves"] == (ref["saves"] if r == 0 else []), (world, r)   # rank 0 writes

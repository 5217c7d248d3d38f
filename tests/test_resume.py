"""Resume from files the REFERENCE wrote (main.py:259-280 --load_model,
Coach.py:187-201): tests/golden/resume_ttt3/ holds the best_gnn.pth.tar checkpoint and the
example history the reference saved after one TicTacToe 3x3 GNN iteration (G9, G7's run).

* CPU: the checkpoint loads with torch.load(weights_only=True) and carries the reference's keys
  and shapes; Coach.loadTrainExamples reads the history (1 iteration, 1320 + 165 examples) and
  sets skipFirstSelfPlay.
* GPU: `main.py --game tictactoe --board_size 3 --use_gnn --numIters 1 --load_model` on those
  files (seeds 1, as the reference's resumed run) skips self-play, trains on the loaded
  history, and its arena W/L/D and written files equal the reference's resumed iteration."""
import json
import os
import random
import shutil

import numpy as np
import pytest

from conftest import GOLDEN

FIX = os.path.join(GOLDEN, "resume_ttt3")


def test_reference_checkpoint_loads_weights_only():
    import torch
    from azhip.weights import gnn_spec, tictactoe_net_spec
    ck = torch.load(os.path.join(FIX, "best_gnn.pth.tar"), map_location="cpu", weights_only=True)
    assert set(ck) == {"state_dict", "gnn"}
    want = dict(tictactoe_net_spec(3, 10))
    assert list(ck["state_dict"]) == list(want)
    for k, shape in want.items():
        assert tuple(ck["state_dict"][k].shape) == tuple(shape), k
    g = dict(gnn_spec(128, 2))
    assert list(ck["gnn"]) == list(g)
    for k, shape in g.items():
        assert tuple(ck["gnn"][k].shape) == tuple(shape), k


def test_reference_examples_history_loads(tmp_path):
    from Coach import Coach
    from tictactoe.TicTacToeGame import TicTacToeGame
    from test_mcts_golden import Args
    coach = Coach.__new__(Coach)
    coach.args = Args(load_folder_file=(FIX, "best_gnn.pth.tar"))
    coach.trainExamplesHistory, coach.skipFirstSelfPlay = [], False
    coach.loadTrainExamples()
    ref = json.load(open(os.path.join(GOLDEN, "resume_ttt3.json")))
    assert coach.skipFirstSelfPlay and len(coach.trainExamplesHistory) == ref["loaded_history"]
    std, gnn = coach.trainExamplesHistory[0]
    assert (len(std), len(gnn)) == (ref["n_std"], ref["n_gnn"])
    game = TicTacToeGame(3)
    b, pi, z = std[0]
    assert np.asarray(b).shape == game.getBoardSize() and len(pi) == game.getActionSize()
    assert len(gnn[0]) == 7


class _Boom:
    def __reduce__(self):
        return (os.system, ("echo should-not-run",))


def test_examples_unpickler_refuses_foreign_globals(tmp_path):
    """loadTrainExamples resolves only numpy / deque globals: a history that names any other
    callable raises instead of running it; a history this Coach saved round-trips."""
    import pickle
    from collections import deque
    from Coach import Coach, ExamplesUnpickler
    from test_mcts_golden import Args
    bad = tmp_path / "bad.pth.tar.examples"
    bad.write_bytes(pickle.dumps([deque([_Boom()])]))
    with open(bad, "rb") as f, pytest.raises(pickle.UnpicklingError, match="os|posix|system"):
        ExamplesUnpickler(f).load()
    coach = Coach.__new__(Coach)
    coach.args = Args(checkpoint=str(tmp_path), load_folder_file=(str(tmp_path), "x.pth.tar"))
    hist = [([(np.zeros((3, 3), np.int64), [0.5, 0.5], 1)],
             [(np.ones((3, 3)), 1, np.full(2, 0.5), np.float32(0.25), np.full(2, 0.5), 0.1, -1)])]
    coach.trainExamplesHistory = hist
    coach.getCheckpointFile = lambda i: "x.pth.tar"
    coach.saveTrainExamples(0)
    coach.trainExamplesHistory, coach.skipFirstSelfPlay = [], False
    coach.loadTrainExamples()
    (std, gnn), = coach.trainExamplesHistory
    assert np.array_equal(std[0][0], hist[0][0][0][0]) and gnn[0][3] == np.float32(0.25)
    # a history pickled with protocol 5 (numpy rebuilds contiguous arrays via _frombuffer)
    p5 = tmp_path / "p5.pth.tar.examples"
    p5.write_bytes(pickle.dumps([deque(hist[0][0]), deque(hist[0][1])], protocol=5))
    with open(p5, "rb") as f:
        got = ExamplesUnpickler(f).load()
    assert np.array_equal(got[0][0][0], hist[0][0][0][0]) and got[1][0][3] == np.float32(0.25)


@pytest.mark.gpu
def test_load_model_resume_matches_reference(tmp_path):
    import torch
    import yaml
    import Arena as A
    import main as M
    ref = json.load(open(os.path.join(GOLDEN, "resume_ttt3.json")))
    cfg = yaml.safe_load(open(os.path.join(M.HERE, "tictactoe", "config.yaml")))
    cfg["training"]["checkpoint_path"] = str(tmp_path)
    cfgp = tmp_path / "config.yaml"
    cfgp.write_text(yaml.safe_dump(cfg))
    folder = tmp_path / "tictactoe"
    folder.mkdir()
    for f in os.listdir(FIX):
        shutil.copy(os.path.join(FIX, f), folder / f)
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    seen = []
    orig = A.Arena.playGames

    def pg(self, num, verbose=False):
        r = orig(self, num, verbose)
        seen.append([int(x) for x in r])
        return r

    A.Arena.playGames = pg
    try:
        coach = M.main(["--game", "tictactoe", "--config", str(cfgp), "--board_size", "3",
                        "--numIters", "1", "--use_gnn", "--load_model"])
    finally:
        A.Arena.playGames = orig
    std, gnn = coach.trainExamplesHistory[0]
    assert (len(coach.trainExamplesHistory), len(std), len(gnn)) == \
        (ref["loaded_history"], ref["n_std"], ref["n_gnn"])
    assert seen[0] == ref["arena_pwins_nwins_draws"], seen
    assert sorted(os.listdir(folder)) == ref["files"]

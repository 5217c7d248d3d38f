"""Self-play / train / gate loop (reference Coach.py:16-201) over this package's MCTS and the
libaz_hip networks.  Same episode semantics (temperature schedule, symmetries, GNN
'sliding-window' examples from MCTS.expand_tree, reward sign per player), same example
history, pickle files and checkpoint names, so --load_model resumes from files either
implementation wrote."""
import logging
import os
import sys
from collections import deque
from pickle import Pickler, Unpickler
from random import shuffle

import numpy as np
from tqdm import tqdm

from Arena import Arena
from MCTS import MCTS
from azhip import dist as D

log = logging.getLogger(__name__)


class ExamplesUnpickler(Unpickler):
    """Loads a `.examples` history (Coach.py:187-201: a list of deques of example tuples of numpy
    arrays, floats and ints) and nothing else.  Only the globals such a file needs resolve --
    numpy array / dtype / scalar reconstruction and collections.deque -- so a file that names
    any other callable raises pickle.UnpicklingError instead of running it."""

    _ALLOWED = {
        ("collections", "deque"),
        ("numpy", "ndarray"), ("numpy", "dtype"),
        ("numpy.core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "scalar"),
        # protocol 5 (Python 3.14's default) rebuilds contiguous arrays from their buffer
        ("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer"),
        ("builtins", "list"), ("builtins", "tuple"), ("builtins", "dict"), ("builtins", "set"),
        ("builtins", "frozenset"), ("builtins", "int"), ("builtins", "float"),
        ("builtins", "bool"), ("builtins", "str"), ("builtins", "bytes"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED or \
                (module == "numpy.dtypes" and name.endswith("DType")):
            return super().find_class(module, name)
        import pickle
        raise pickle.UnpicklingError(f".examples file names {module}.{name}: not an example "
                                     "history (only numpy arrays, scalars and deques load)")


def _flag(args, name, default=False):
    try:
        return args[name] if isinstance(args, dict) else getattr(args, name)
    except (KeyError, AttributeError):
        return default


def _native_ok(game):
    """The native engine covers Connect4Game / TicTacToeGame boards up to 64 cells."""
    try:
        import mcts_native
        mcts_native.game_kind(game)
        mcts_native.lib()
        return True
    except (ValueError, RuntimeError, OSError):
        return False


def episode_g(game, args, mcts, rng=None):
    """Coach.py:27-79 as a search generator (see MCTS.py): one self-play game ->
    (std_examples, gnn_examples), with the final result r signed per example by whether its
    player is the one to move at the end.  `rng` (default: the global np.random stream, as the
    reference) draws the moves; mcts.rng draws the temp-0 tie-breaks."""
    choice = (np.random if rng is None else rng).choice
    use_gnn = _flag(args, "use_gnn")
    examples, gnn_examples = [], []
    board = game.getInitBoard()
    cur = 1
    step = 0
    while True:
        step += 1
        canonical = game.getCanonicalForm(board, cur)
        temp = int(step < args.tempThreshold)
        pi = yield from mcts.getActionProb_g(canonical, temp=temp)
        sym = game.getSymmetries(canonical, pi)
        examples.extend([b, cur, p, None] for b, p in sym)
        if use_gnn:
            nodes = yield from mcts.expand_tree_g(canonical, expand_by=_flag(args, "expand_by", 5))
            for s, (ipi, iv, epi, ev) in nodes.items():
                for b, _ in sym:
                    if game.stringRepresentation(b) == s:
                        gnn_examples.append([b, cur, ipi, iv, epi, ev, None])
                        break
        action = choice(len(pi), p=pi)
        board, cur = game.getNextState(board, cur, action)
        r = game.getGameEnded(board, cur)
        if r != 0:
            def sign(p):
                return r * ((-1) ** (p != cur))
            std = [(x[0], x[2], sign(x[1])) for x in examples]
            if use_gnn and gnn_examples:
                return std, [(x[0], x[1], x[2], x[3], x[4], x[5], sign(x[1]))
                             for x in gnn_examples]
            return std, []


class Coach:
    def __init__(self, game, nnet, args):
        self.game = game
        self.nnet = nnet
        self.pnet = self.nnet.__class__(self.game, args)   # the competitor (Coach.py:21)
        self.args = args
        self.mcts = MCTS(self.game, self.nnet, self.args)
        self.trainExamplesHistory = []
        self.skipFirstSelfPlay = False

    def executeEpisode(self):
        """Coach.py:27-79: one self-play game -> (std_examples, gnn_examples)."""
        return self.mcts.drive(episode_g(self.game, self.args, self.mcts))

    def getCheckpointFile(self, iteration):
        return f"checkpoint_{iteration}" + ("_gnn" if _flag(self.args, "use_gnn") else "") + \
            ".pth.tar"

    def selfPlay(self):
        """One iteration's self-play (Coach.py:95-100) -> [(std, gnn)] in episode order.

        parallel_games <= 1 on one rank: the reference's sequential loop on the global RNG.
        Otherwise lock-step batched games, episode e on rank e mod P with its own RandomState:
        whole episodes in the native engine (selfplay.play_episodes_engine; args.selfplay_engine
        = "python" selects the Python search generators instead); results gathered on every
        rank and ordered by episode, so every P and G produce the same examples."""
        n = self.args.numEps
        parallel = int(_flag(self.args, "parallel_games", 1) or 1)
        world, rank = D.world_rank()
        if parallel <= 1 and world == 1:
            out = []
            for _ in tqdm(range(n), desc="Self Play"):
                self.mcts = MCTS(self.game, self.nnet, self.args)
                out.append(self.executeEpisode())
            return out
        from selfplay import episode_seeds, play_episodes, play_episodes_engine
        base = D.broadcast_int(np.random.randint(0, 2 ** 31 - 1))
        seeds = episode_seeds(base, range(n))
        mine = D.my_episodes(n, world, rank)
        if _flag(self.args, "selfplay_engine", "native") == "native" and _native_ok(self.game):
            local = play_episodes_engine(self.game, self.nnet, self.args, mine, seeds,
                                         parallel_games=max(1, parallel))
        else:
            local = play_episodes(self.game, self.nnet, self.args, mine, seeds,
                                  parallel_games=max(1, parallel))
        allr = D.gather_episodes(local)
        return [allr[e] for e in range(n)]

    def _is_writer(self):
        return D.world_rank()[1] == 0

    def _barrier(self):
        if D.dist_ok():
            import torch.distributed as dist
            dist.barrier()

    def learn(self):
        """Coach.py:87-176.  Under torch.distributed every rank runs this loop on identical
        data (host RNGs synchronised here); only rank 0 writes files."""
        use_gnn = _flag(self.args, "use_gnn")
        if D.dist_ok():        # any process group, world size 1 included: same RNG use for any P
            D.sync_host_rngs()
        for i in range(1, self.args.numIters + 1):
            log.info(f"Starting Iter #{i} ...")
            if not self.skipFirstSelfPlay or i > 1:
                it_std = deque([], maxlen=self.args.maxlenOfQueue)
                it_gnn = deque([], maxlen=self.args.maxlenOfQueue)
                for std, gnn in self.selfPlay():
                    it_std += std
                    if gnn:
                        it_gnn += gnn
                self.trainExamplesHistory.append((it_std, it_gnn))
            if len(self.trainExamplesHistory) > self.args.numItersForTrainExamplesHistory:
                log.warning("Removing the oldest entry in trainExamples. "
                            f"len(trainExamplesHistory) = {len(self.trainExamplesHistory)}")
                self.trainExamplesHistory.pop(0)
            if self._is_writer():
                self.saveTrainExamples(i - 1)

            trainExamples, gnnExamples = [], []
            for std_ex, gnn_ex in self.trainExamplesHistory:
                trainExamples.extend(std_ex)
                if gnn_ex:
                    gnnExamples.extend(gnn_ex)
            shuffle(trainExamples)
            if gnnExamples:
                shuffle(gnnExamples)

            temp = "temp.pth.tar"
            if self._is_writer():
                self.nnet.save_checkpoint(folder=self.args.checkpoint, filename=temp)
            self._barrier()
            self.pnet.load_checkpoint(folder=self.args.checkpoint, filename=temp)
            native_arena = (_flag(self.args, "selfplay_engine", "native") == "native"
                            and _native_ok(self.game))
            if native_arena:
                from mcts_native import ArenaPlayer
                pplayer = ArenaPlayer(self.game, self.pnet, self.args)
            else:
                pmcts = MCTS(self.game, self.pnet, self.args)
                pplayer = lambda x: np.argmax(pmcts.getActionProb(x, temp=0))  # noqa: E731
            if use_gnn and gnnExamples:
                log.info(f"Training with {len(trainExamples)} standard examples and "
                         f"{len(gnnExamples)} GNN examples")
                self.nnet.train(trainExamples, gnnExamples)
            else:
                self.nnet.train(trainExamples)
            if native_arena:
                nplayer = ArenaPlayer(self.game, self.nnet, self.args)
            else:
                nmcts = MCTS(self.game, self.nnet, self.args)
                nplayer = lambda x: np.argmax(nmcts.getActionProb(x, temp=0))  # noqa: E731

            log.info("PITTING AGAINST PREVIOUS VERSION")
            # Arena.py:249-291 with the reference's per-iteration MCTS objects (one tree per
            # player for all games); the native players run the same searches in C++
            arena = Arena(pplayer, nplayer, self.game)
            pwins, nwins, draws = arena.playGames(self.args.arenaCompare)
            log.info("NEW/PREV WINS : %d / %d ; DRAWS : %d" % (nwins, pwins, draws))
            if i == 1:
                log.info("FIRST ITERATION: SAVING AS BEST MODEL")
                accept = True
            else:
                accept = (pwins + nwins > 0) and \
                    (float(nwins) / (pwins + nwins) >= self.args.updateThreshold)
            if not accept:
                log.info("REJECTING NEW MODEL")
                self.nnet.load_checkpoint(folder=self.args.checkpoint, filename=temp)
            else:
                log.info("ACCEPTING NEW MODEL")
                best = "best_gnn.pth.tar" if use_gnn else "best.pth.tar"
                it_name = f"checkpoint_{i}_gnn.pth.tar" if use_gnn else f"checkpoint_{i}.pth.tar"
                if self._is_writer():
                    self.nnet.save_checkpoint(folder=self.args.checkpoint, filename=it_name)
                    self.nnet.save_checkpoint(folder=self.args.checkpoint, filename=best)
            self._barrier()

    def saveTrainExamples(self, iteration):
        folder = self.args.checkpoint
        if not os.path.exists(folder):
            os.makedirs(folder)
        filename = os.path.join(folder, self.getCheckpointFile(iteration) + ".examples")
        with open(filename, "wb+") as f:
            Pickler(f).dump(self.trainExamplesHistory)

    def loadTrainExamples(self):
        """Coach.py:187-201.  The .examples file is a pickle this program (or the reference)
        wrote itself; do not point it at untrusted files."""
        modelFile = os.path.join(self.args.load_folder_file[0], self.args.load_folder_file[1])
        examplesFile = modelFile + ".examples"
        if not os.path.isfile(examplesFile):
            log.warning(f'File "{examplesFile}" with trainExamples not found!')
            r = input("Continue? [y|n]")
            if r != "y":
                sys.exit()
        else:
            log.info("File with trainExamples found. Loading it...")
            with open(examplesFile, "rb") as f:
                self.trainExamplesHistory = ExamplesUnpickler(f).load()
            log.info("Loading done!")
            self.skipFirstSelfPlay = True

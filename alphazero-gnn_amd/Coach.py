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

log = logging.getLogger(__name__)


def _flag(args, name, default=False):
    try:
        return args[name] if isinstance(args, dict) else getattr(args, name)
    except (KeyError, AttributeError):
        return default


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
        """Coach.py:27-79: one self-play game -> (std_examples, gnn_examples) with the final
        result r signed per example by whether its player is the one to move at the end."""
        use_gnn = _flag(self.args, "use_gnn")
        examples, gnn_examples = [], []
        board = self.game.getInitBoard()
        self.curPlayer = 1
        step = 0
        while True:
            step += 1
            canonical = self.game.getCanonicalForm(board, self.curPlayer)
            temp = int(step < self.args.tempThreshold)
            pi = self.mcts.getActionProb(canonical, temp=temp)
            sym = self.game.getSymmetries(canonical, pi)
            examples.extend([b, self.curPlayer, p, None] for b, p in sym)
            if use_gnn:
                nodes = self.mcts.expand_tree(canonical,
                                              expand_by=_flag(self.args, "expand_by", 5))
                for s, (ipi, iv, epi, ev) in nodes.items():
                    for b, _ in sym:
                        if self.game.stringRepresentation(b) == s:
                            gnn_examples.append([b, self.curPlayer, ipi, iv, epi, ev, None])
                            break
            action = np.random.choice(len(pi), p=pi)
            board, self.curPlayer = self.game.getNextState(board, self.curPlayer, action)
            r = self.game.getGameEnded(board, self.curPlayer)
            if r != 0:
                def sign(p):
                    return r * ((-1) ** (p != self.curPlayer))
                std = [(x[0], x[2], sign(x[1])) for x in examples]
                if use_gnn and gnn_examples:
                    return std, [(x[0], x[1], x[2], x[3], x[4], x[5], sign(x[1]))
                                 for x in gnn_examples]
                return std, []

    def getCheckpointFile(self, iteration):
        return f"checkpoint_{iteration}" + ("_gnn" if _flag(self.args, "use_gnn") else "") + \
            ".pth.tar"

    def learn(self):
        """Coach.py:87-176."""
        use_gnn = _flag(self.args, "use_gnn")
        for i in range(1, self.args.numIters + 1):
            log.info(f"Starting Iter #{i} ...")
            if not self.skipFirstSelfPlay or i > 1:
                it_std = deque([], maxlen=self.args.maxlenOfQueue)
                it_gnn = deque([], maxlen=self.args.maxlenOfQueue)
                for _ in tqdm(range(self.args.numEps), desc="Self Play"):
                    self.mcts = MCTS(self.game, self.nnet, self.args)
                    std, gnn = self.executeEpisode()
                    it_std += std
                    if gnn:
                        it_gnn += gnn
                self.trainExamplesHistory.append((it_std, it_gnn))
            if len(self.trainExamplesHistory) > self.args.numItersForTrainExamplesHistory:
                log.warning("Removing the oldest entry in trainExamples. "
                            f"len(trainExamplesHistory) = {len(self.trainExamplesHistory)}")
                self.trainExamplesHistory.pop(0)
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
            self.nnet.save_checkpoint(folder=self.args.checkpoint, filename=temp)
            self.pnet.load_checkpoint(folder=self.args.checkpoint, filename=temp)
            pmcts = MCTS(self.game, self.pnet, self.args)
            if use_gnn and gnnExamples:
                log.info(f"Training with {len(trainExamples)} standard examples and "
                         f"{len(gnnExamples)} GNN examples")
                self.nnet.train(trainExamples, gnnExamples)
            else:
                self.nnet.train(trainExamples)
            nmcts = MCTS(self.game, self.nnet, self.args)

            log.info("PITTING AGAINST PREVIOUS VERSION")
            arena = Arena(lambda x: np.argmax(pmcts.getActionProb(x, temp=0)),
                          lambda x: np.argmax(nmcts.getActionProb(x, temp=0)), self.game)
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
                self.nnet.save_checkpoint(folder=self.args.checkpoint, filename=it_name)
                self.nnet.save_checkpoint(folder=self.args.checkpoint, filename=best)

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
                self.trainExamplesHistory = Unpickler(f).load()
            log.info("Loading done!")
            self.skipFirstSelfPlay = True

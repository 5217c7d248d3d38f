"""Two-player arena (reference Arena.py:106-152, 249-291): pits two action functions,
each starting half of the games.  The single-player (FrozenLake) branch of the reference is
out of scope."""
import logging

from tqdm import tqdm

log = logging.getLogger(__name__)


class Arena:
    def __init__(self, player1, player2, game, display=None):
        self.player1 = player1
        self.player2 = player2
        self.game = game
        self.display = display
        self.is_single_player = hasattr(self.game, "is_two_player") and not self.game.is_two_player

    def playGameForTwoPlayer(self, verbose=False):
        """One game; returns +1 if player1 won, -1 if player2 won, the draw value otherwise
        (curPlayer * getGameEnded(board, curPlayer), Arena.py:152)."""
        players = {1: self.player1, -1: self.player2}
        cur = 1
        board = self.game.getInitBoard()
        it = 0
        for p in (self.player2, self.player1):
            if hasattr(p, "startGame"):
                p.startGame()
        while self.game.getGameEnded(board, cur) == 0:
            it += 1
            if verbose:
                assert self.display
                print("Turn ", str(it), "Player ", str(cur))
                self.display(board)
            canonical = self.game.getCanonicalForm(board, cur)
            action = players[cur](canonical)
            valids = self.game.getValidMoves(self.game.getCanonicalForm(board, cur), 1)
            if valids[action] == 0:
                log.error(f"Action {action} is not valid!")
                log.debug(f"valids = {valids}")
                assert valids[action] > 0
            opponent = players[-cur]
            if hasattr(opponent, "notify"):
                opponent.notify(board, action)
            board, cur = self.game.getNextState(board, cur, action)
        for p in (self.player2, self.player1):
            if hasattr(p, "endGame"):
                p.endGame()
        if verbose:
            assert self.display
            print("Game over: Turn ", str(it), "Result ", str(self.game.getGameEnded(board, 1)))
            self.display(board)
        return cur * self.game.getGameEnded(board, cur)

    def playGamesForTwoPlayer(self, num, verbose=False):
        """num/2 games with player1 first, then num/2 with the roles swapped
        -> (player1 wins, player2 wins, draws) counted against the ORIGINAL player1."""
        num = int(num / 2)
        one = two = draws = 0
        for _ in tqdm(range(num), desc="Arena.playGames (Two-Player) (1)"):
            r = self.playGameForTwoPlayer(verbose=verbose)
            if r == 1:
                one += 1
            elif r == -1:
                two += 1
            else:
                draws += 1
        self.player1, self.player2 = self.player2, self.player1
        for _ in tqdm(range(num), desc="Arena.playGames (Two-Player) (2)"):
            r = self.playGameForTwoPlayer(verbose=verbose)
            if r == -1:
                one += 1
            elif r == 1:
                two += 1
            else:
                draws += 1
        return one, two, draws

    def playGames(self, num, verbose=False):
        if self.is_single_player:
            raise NotImplementedError("single-player arena (FrozenLake) is out of scope")
        return self.playGamesForTwoPlayer(num, verbose)

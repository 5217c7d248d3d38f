"""Game registry (reference register.py:1-79): name -> (Game, standard net, GNN net).
FrozenLake (gymnasium, no GNN) is not registered: out of scope."""

GAME_REGISTRY = {}


def register_game(name, game_class, standard_nnet_class, gnn_nnet_class=None):
    GAME_REGISTRY[name] = (game_class, standard_nnet_class, gnn_nnet_class)


def get_game(name, use_gnn=False):
    """(game_class, nnet_class); ValueError for an unknown game or a missing GNN version."""
    if name not in GAME_REGISTRY:
        raise ValueError(f"Game '{name}' not found in registry. Available games: "
                         f"{list(GAME_REGISTRY.keys())}")
    game_class, standard, gnn = GAME_REGISTRY[name]
    if use_gnn:
        if gnn is None:
            raise ValueError(f"GNN version of '{name}' is not implemented")
        return (game_class, gnn)
    return (game_class, standard)


def list_games():
    return list(GAME_REGISTRY.keys())


def has_gnn_version(name):
    return name in GAME_REGISTRY and GAME_REGISTRY[name][2] is not None


from tictactoe.TicTacToeGame import TicTacToeGame  # noqa: E402
from tictactoe.TicTacToeNet import TicTacToeNNetWrapper  # noqa: E402
from tictactoe.TicTacToeGNN import TicTacToeGNNWrapper  # noqa: E402

register_game("tictactoe", TicTacToeGame, TicTacToeNNetWrapper, TicTacToeGNNWrapper)

from connect4.Connect4Game import Connect4Game  # noqa: E402
from connect4.Connect4Net import Connect4NNetWrapper  # noqa: E402
from connect4.Connect4GNN import Connect4GNNWrapper  # noqa: E402

register_game("connect4", Connect4Game, Connect4NNetWrapper, Connect4GNNWrapper)

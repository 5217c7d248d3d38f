"""Entry point with the reference's CLI and config.yaml surface (reference main.py:1-58,140-293).

    python main.py --game connect4 [--use_gnn] [--gnn_layers 2] [--config connect4/config.yaml]
                   [--board_size N] [--numIters N] [--numMCTSSims N] [--load_model] [--pit_gnn]

YAML sections are flattened into one namespace; --use_gnn / --gnn_layers always override the
YAML (main.py:217-218), the three numeric overrides only when given.  Checkpoints go to
<checkpoint_path>/<game>/ with the reference's file names.

MI355X additions (absent from the reference; defaults reproduce its behaviour):
    --parallel_games G       lock-step batched self-play with G concurrent games (selfplay.py)
    --train_parallel MODE    "replicas" | "allreduce" (azhip/dist.py) under torch.distributed
    multi-GPU: python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 main.py ...
               (one rank per GPU, backend nccl = RCCL; episodes sharded by index)
"""
import argparse
import logging
import os
import sys

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import hostcpu  # noqa: E402

hostcpu.engine_omp_defaults()    # before the OpenMP runtime starts (torch, the engine)

from Arena import Arena  # noqa: E402
from Coach import Coach  # noqa: E402
from MCTS import MCTS  # noqa: E402
from register import get_game, has_gnn_version, list_games  # noqa: E402

log = logging.getLogger(__name__)


class dotdict(dict):
    def __getattr__(self, name):
        return self[name]

    def __setattr__(self, name, value):
        self[name] = value


def load_config(path):
    with open(path) as f:
        return yaml.safe_load(f)


def config_to_args(config):
    """main.py:30-43: flatten every section; keep checkpoint / checkpoint_path aliases."""
    args = dotdict({})
    for section in config:
        for k, v in (config[section] or {}).items():
            args[k] = v
    if "checkpoint_path" in args and "checkpoint" not in args:
        args.checkpoint = args.checkpoint_path
    elif "checkpoint" in args and "checkpoint_path" not in args:
        args.checkpoint_path = args.checkpoint
    return args


def get_checkpoint_path(game_name, filename, use_gnn=False, base_path="./checkpoints"):
    """main.py:45-58: (<base>/<game>, best[_gnn].pth.tar)."""
    folder = os.path.join(base_path, game_name)
    if use_gnn and not filename.endswith("_gnn.pth.tar"):
        filename = filename.replace(".pth.tar", "_gnn.pth.tar") if filename.endswith(".pth.tar") \
            else f"{filename}_gnn.pth.tar"
    elif not filename.endswith(".pth.tar"):
        filename = f"{filename}.pth.tar"
    return folder, filename


def create_game_instance(GameClass, args):
    """main.py:140-156 for the two registered games."""
    if args.game == "tictactoe":
        return GameClass(n=args.board_size)
    if args.game == "connect4":
        return GameClass(board_size=args.board_size)
    return GameClass(**{k: v for k, v in args.items()
                        if k in GameClass.__init__.__code__.co_varnames})


def pit_gnn_vs_regular(game_name, args):
    """main.py:60-138: best_gnn.pth.tar against best.pth.tar over arenaCompare games."""
    if not has_gnn_version(game_name):
        log.error(f"Game '{game_name}' does not have a GNN version implemented")
        return None
    folder = os.path.join(args.checkpoint_path, game_name)
    for fname, hint in (("best.pth.tar", ""), ("best_gnn.pth.tar", " --use_gnn")):
        if not os.path.exists(os.path.join(folder, fname)):
            log.error(f"Model not found at {os.path.join(folder, fname)}; "
                      f"run: python main.py --game {game_name}{hint}")
            sys.exit(1)
    GameClass, Reg = get_game(game_name, use_gnn=False)
    _, Gnn = get_game(game_name, use_gnn=True)
    game = create_game_instance(GameClass, args)
    reg_args, gnn_args = dotdict(args.copy()), dotdict(args.copy())
    reg_args.use_gnn, gnn_args.use_gnn = False, True
    reg, gnn = Reg(game, reg_args), Gnn(game, gnn_args)
    reg.load_checkpoint(folder, "best.pth.tar")
    gnn.load_checkpoint(folder, "best_gnn.pth.tar")
    rm, gm = MCTS(game, reg, reg_args), MCTS(game, gnn, gnn_args)
    arena = Arena(lambda x: np.argmax(gm.getActionProb(x, temp=0)),
                  lambda x: np.argmax(rm.getActionProb(x, temp=0)), game)
    g, r, d = arena.playGames(args.arenaCompare)
    log.info("GNN/REGULAR WINS : %d / %d ; DRAWS : %d" % (g, r, d))
    return g, r, d


def parse(argv=None):
    p = argparse.ArgumentParser(description="AlphaZero for Multiple Games (MI355X)")
    p.add_argument("--game", type=str, required=True,
                   help=f"Game to train. Available games: {', '.join(list_games())}")
    p.add_argument("--config", type=str, default=None,
                   help="Path to configuration file (default: <game>/config.yaml)")
    p.add_argument("--load_model", action="store_true")
    p.add_argument("--use_gnn", action="store_true")
    p.add_argument("--gnn_layers", type=int, default=2)
    p.add_argument("--pit_gnn", action="store_true")
    p.add_argument("--board_size", type=int)
    p.add_argument("--numIters", type=int)
    p.add_argument("--numMCTSSims", type=int)
    p.add_argument("--parallel_games", type=int, default=None)
    p.add_argument("--train_parallel", choices=["replicas", "allreduce"], default=None)
    return p.parse_args(argv)


def build_args(a):
    """main.py:181-236: config file + CLI overrides -> dotdict (and the checkpoint folder)."""
    if a.game not in list_games():
        log.error(f"Game '{a.game}' not found in registry. Available games: {list_games()}")
        sys.exit(1)
    if a.use_gnn and not has_gnn_version(a.game):
        log.error(f"GNN version of '{a.game}' is not implemented")
        sys.exit(1)
    cfg_path = a.config or os.path.join(HERE, a.game, "config.yaml")
    try:
        config = load_config(cfg_path)
    except Exception as e:
        log.error(f"Error loading configuration: {e}")
        sys.exit(1)
    args = config_to_args(config)
    for k in ("board_size", "numIters", "numMCTSSims", "parallel_games", "train_parallel"):
        if getattr(a, k) is not None:
            args[k] = getattr(a, k)
    args.use_gnn = a.use_gnn
    args.gnn_layers = a.gnn_layers
    args.game = a.game
    args.load_model = a.load_model
    folder, best = get_checkpoint_path(a.game, "best", use_gnn=a.use_gnn,
                                       base_path=args.checkpoint_path)
    os.makedirs(folder, exist_ok=True)
    args.checkpoint = folder
    args.load_folder_file = (folder, best)
    return args


def init_distributed():
    """One rank per GPU when launched by torch.distributed.run (RANK/WORLD_SIZE set)."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))


def main(argv=None):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    a = parse(argv)
    args = build_args(a)
    init_distributed()
    if a.pit_gnn:
        return pit_gnn_vs_regular(a.game, args)
    GameClass, NNetClass = get_game(a.game, use_gnn=a.use_gnn)
    log.info(f"Creating {a.game} game with board size {args.board_size}")
    game = create_game_instance(GameClass, args)
    nnet = NNetClass(game, args)
    if args.load_model:
        try:
            nnet.load_checkpoint(*args.load_folder_file)
        except Exception as e:
            log.warning(f"Could not load model checkpoint: {e}; starting with a new model")
    coach = Coach(game, nnet, args)
    if args.load_model:
        try:
            coach.loadTrainExamples()
        except Exception as e:
            log.warning(f"Could not load training examples: {e}")
    try:
        coach.learn()
    except KeyboardInterrupt:
        log.warning("Training interrupted by user")
        _, fname = get_checkpoint_path(a.game, "interrupted", use_gnn=a.use_gnn)
        nnet.save_checkpoint(args.checkpoint, fname)
    return coach


if __name__ == "__main__":
    main()

"""azchess -- MI355X-native self-play engine for AlexandreGac/alphazero-chess' MCTS+NN hot path.

Host-side mirror of the reference's module surface (chess.rs, agent.rs, tree.rs,
training.rs, parameters.rs) over the C-ABI of libaz.so (include/az.h).
"""
from . import _lib, parameters
from .agent import AlphaZero, load_model, load_mpk, num_params, random_weights, save_mpk
from .chess import (GameResult, GameState, IllegalMove, Position, index_to_move, move_to_index, play_move,
                    to_tensor)
from .memory import ReplayBuffer, TrainingSample
from .training import (EpisodeStep, SelfPlay, Trainer, comm_unique_id, get_cyclical_lr, process_batch,
                       run_all_episodes, run_episode, train)
from .tree import BatchedSearch, MCTree, make_cfg
from .validation import EvaluationResult, Player, compute_elo_rankings, compute_elos, evaluate

__all__ = ["AlphaZero", "load_model", "load_mpk", "save_mpk", "num_params", "random_weights", "GameResult", "GameState", "IllegalMove", "Position",
           "index_to_move", "move_to_index", "play_move", "to_tensor", "EpisodeStep", "SelfPlay", "Trainer", "comm_unique_id",
           "get_cyclical_lr", "process_batch", "train", "ReplayBuffer", "TrainingSample",
           "run_all_episodes", "run_episode", "BatchedSearch", "MCTree", "make_cfg", "parameters", "EvaluationResult", "Player",
           "compute_elo_rankings", "compute_elos", "evaluate"]

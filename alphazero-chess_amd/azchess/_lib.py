"""ctypes binding of libaz.so (include/az.h).

The product path is libaz.so only: if the library is missing this module raises at import
time -- there is no Python or CPU fallback for any compute entry point.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# AZ_LIB selects an alternative in-tree build of the same ABI (kernel-variant A/B runs)
LIB_PATH = os.environ.get("AZ_LIB") or os.path.join(_HERE, "libaz.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

ACTION_SPACE = 4096
MAX_MOVES = 256
ONGOING, DRAW, WHITE_WINS, BLACK_WINS, ILLEGAL = 0, 1, 2, 3, -1
DTYPE_F32, DTYPE_BF16 = 0, 1
EVAL_NET, EVAL_SYNTHETIC, EVAL_CALLBACK = 0, 1, 2


class AzPos(C.Structure):
    _fields_ = [("bb", C.c_uint64 * 8), ("turn", C.c_uint8), ("castling", C.c_uint8), ("ep", C.c_uint8),
                ("flags", C.c_uint8), ("halfmoves", C.c_uint16), ("fullmoves", C.c_uint16),
                ("rep_key", C.c_uint64)]


# the same 80-byte record as a numpy dtype (batched test data)
POS_DTYPE = np.dtype({
    "names": ["bb", "turn", "castling", "ep", "flags", "halfmoves", "fullmoves", "rep_key"],
    "formats": [("<u8", (8,)), "u1", "u1", "u1", "u1", "<u2", "<u2", "<u8"],
    "offsets": [0, 64, 65, 66, 67, 68, 70, 72], "itemsize": 80})


class AzNetDesc(C.Structure):
    _fields_ = [("blocks", C.c_int), ("filters", C.c_int), ("dtype", C.c_int)]


class AzSearchCfg(C.Structure):
    _fields_ = [("games", C.c_int), ("sims", C.c_int), ("c_puct", C.c_float), ("dir_alpha", C.c_float),
                ("dir_eps", C.c_float), ("temp_moves", C.c_int), ("noise", C.c_int), ("seed", C.c_uint64),
                ("evaluator", C.c_int), ("continuous", C.c_int), ("record_evals", C.c_int),
                ("eval_log_cap", C.c_int), ("cache_capacity", C.c_int)]


class AzEpisodeStep(C.Structure):
    _fields_ = [("game_id", C.c_int32), ("ply", C.c_int32), ("action", C.c_int32), ("search_depth", C.c_int32),
                ("final_value", C.c_float), ("result", C.c_int32), ("nvis", C.c_int32), ("state", AzPos),
                ("vis_idx", C.c_uint16 * 224), ("vis_n", C.c_uint16 * 224)]


class AzSearchStats(C.Structure):
    _fields_ = [("sims", C.c_int64), ("evals", C.c_int64), ("terminal_leaves", C.c_int64),
                ("games_finished", C.c_int64), ("moves", C.c_int64), ("max_depth_sum", C.c_int64),
                ("cache_hits", C.c_int64), ("cache_misses", C.c_int64), ("overflow", C.c_int64),
                ("max_nodes", C.c_int64), ("max_edges", C.c_int64), ("node_cap", C.c_int64), ("edge_cap", C.c_int64)]


class AzTiming(C.Structure):
    _fields_ = [("conv_ms", C.c_double), ("conv_launches", C.c_int64), ("conv_flop", C.c_double),
                ("tower_ms", C.c_double), ("tower_flop", C.c_double),
                ("select_ms", C.c_double), ("select_launches", C.c_int64), ("select_bytes", C.c_double),
                ("expand_ms", C.c_double), ("encode_ms", C.c_double), ("heads_ms", C.c_double),
                ("backup_ms", C.c_double), ("sim_step_ms", C.c_double), ("sim_steps", C.c_int64),
                ("rows", C.c_int64)]


# az_eval_fn (include/az.h): int (*)(void* ctx, const az_pos*, int n, float* policy, float* value)
EVAL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(AzPos), C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float))

# az_allreduce_fn (include/az.h): int (*)(void* ctx, float* buf, size_t n)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.c_size_t)

# every symbol include/az.h declares: (name, restype, argtypes)
P = C.POINTER
SIGNATURES = [
    ("az_last_error", C.c_char_p, []),
    ("az_version", C.c_int, []),
    ("az_device_count", C.c_int, [P(C.c_int)]),
    ("az_device_synchronize", C.c_int, [C.c_int]),
    ("az_pos_startpos", C.c_int, [P(AzPos)]),
    ("az_pos_from_fen", C.c_int, [C.c_char_p, P(AzPos)]),
    ("az_pos_to_fen", C.c_int, [P(AzPos), C.c_char_p, C.c_int]),
    ("az_pos_fen_key", C.c_uint64, [P(AzPos)]),
    ("az_pos_legal_indices", C.c_int, [P(AzPos), P(C.c_int32), C.c_int]),
    ("az_pos_play_index", C.c_int, [P(AzPos), C.c_int32, P(AzPos)]),
    ("az_move_to_index", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("az_pos_outcome", C.c_int, [P(AzPos)]),
    ("az_pos_encode", C.c_int, [P(AzPos), P(C.c_float)]),
    ("az_game_create", C.c_int, [P(C.c_void_p)]),
    ("az_game_clone", C.c_int, [C.c_void_p, P(C.c_void_p)]),
    ("az_game_destroy", C.c_int, [C.c_void_p]),
    ("az_game_position", C.c_int, [C.c_void_p, P(AzPos)]),
    ("az_game_history", C.c_int, [C.c_void_p, P(C.c_int32), C.c_int]),
    ("az_game_play", C.c_int, [C.c_void_p, C.c_int32]),
    ("az_net_num_params", C.c_size_t, [C.c_int, C.c_int]),
    ("az_net_create", C.c_int, [P(AzNetDesc), P(C.c_float), C.c_size_t, C.c_int, P(C.c_void_p)]),
    ("az_net_destroy", C.c_int, [C.c_void_p]),
    ("az_net_tower_kernel", C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    ("az_net_load_mpk", C.c_int, [C.c_char_p, C.c_int, C.c_int, P(C.c_float), C.c_size_t]),
    ("az_net_save_mpk", C.c_int, [C.c_char_p, C.c_int, C.c_int, P(C.c_float), C.c_size_t]),
    ("az_net_forward", C.c_int, [C.c_void_p, P(C.c_float), C.c_int, P(C.c_float), P(C.c_float)]),
    ("az_net_forward_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("az_search_default_cfg", C.c_int, [P(AzSearchCfg)]),
    ("az_search_create", C.c_int, [C.c_void_p, P(AzSearchCfg), C.c_int, P(C.c_void_p)]),
    ("az_search_destroy", C.c_int, [C.c_void_p]),
    ("az_search_set_evaluator", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("az_search_set_roots", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32), P(C.c_int32), P(C.c_int32),
                                      C.c_int]),
    ("az_search_set_roots_from", C.c_int, [C.c_void_p, P(AzPos), P(C.c_int32), P(C.c_int32), P(C.c_int32),
                                           P(C.c_int32), C.c_int]),
    ("az_search_run", C.c_int, [C.c_void_p, P(C.c_float), P(C.c_uint32), P(C.c_int32)]),
    ("az_search_read_roots", C.c_int, [C.c_void_p, P(C.c_float), P(C.c_uint32), P(C.c_int32)]),
    ("az_search_advance", C.c_int, [C.c_void_p, P(C.c_int32), C.c_int, P(C.c_int32)]),
    ("az_selfplay_reset", C.c_int, [C.c_void_p]),
    ("az_selfplay_step", C.c_int, [C.c_void_p, P(C.c_int), P(C.c_int)]),
    ("az_selfplay_run_sims", C.c_int, [C.c_void_p, C.c_int, P(C.c_int), P(C.c_int), P(C.c_int)]),
    ("az_selfplay_drain", C.c_int, [C.c_void_p, P(AzEpisodeStep), C.c_int]),
    ("az_search_stats_get", C.c_int, [C.c_void_p, P(AzSearchStats)]),
    ("az_search_persistent", C.c_int, [C.c_void_p]),
    ("az_search_eval_log", C.c_int, [C.c_void_p, P(C.c_int64), P(C.c_int64), P(C.c_uint64), P(C.c_float),
                                     P(C.c_int32), P(C.c_int32), P(C.c_float)]),
    ("az_search_timing", C.c_int, [C.c_void_p, P(AzTiming), C.c_int, C.c_int]),
    ("az_cyclical_lr", C.c_double, [C.c_int]),
    ("az_trainer_create", C.c_int, [C.c_int, C.c_int, P(C.c_float), C.c_size_t, C.c_int, C.c_int,
                                    P(C.c_void_p)]),
    ("az_trainer_destroy", C.c_int, [C.c_void_p]),
    ("az_trainer_compute_grads", C.c_int, [C.c_void_p, P(C.c_float), P(C.c_float), P(C.c_float), C.c_int,
                                           P(C.c_float)]),
    ("az_trainer_apply", C.c_int, [C.c_void_p, C.c_double]),
    ("az_trainer_step", C.c_int, [C.c_void_p, P(C.c_float), P(C.c_float), P(C.c_float), C.c_int, C.c_double,
                                  P(C.c_float)]),
    ("az_trainer_get_params", C.c_int, [C.c_void_p, P(C.c_float), C.c_size_t]),
    ("az_trainer_get_grads", C.c_int, [C.c_void_p, P(C.c_float), C.c_size_t]),
    ("az_trainer_relu_output", C.c_int, [C.c_void_p, C.c_int, P(C.c_float), C.c_size_t]),
    ("az_trainer_timing", C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double), P(C.c_int64), C.c_int]),
    ("az_comm_unique_id", C.c_int, [C.c_void_p, C.c_int]),
    ("az_replay_create", C.c_int, [C.c_int, P(C.c_void_p)]),
    ("az_replay_destroy", C.c_int, [C.c_void_p]),
    ("az_replay_len", C.c_int, [C.c_void_p]),
    ("az_replay_add", C.c_int, [C.c_void_p, P(AzEpisodeStep)]),
    ("az_replay_add_many", C.c_int, [C.c_void_p, P(AzEpisodeStep), C.c_int]),
    ("az_replay_add_dense", C.c_int, [C.c_void_p, P(AzPos), P(C.c_float), C.c_float]),
    ("az_replay_sample", C.c_int, [C.c_void_p, C.c_int, C.c_uint64, P(C.c_float), P(C.c_float), P(C.c_float),
                                   P(AzPos)]),
    ("az_replay_save", C.c_int, [C.c_void_p, C.c_char_p]),
    ("az_replay_load", C.c_int, [C.c_char_p, C.c_int, P(C.c_void_p)]),
    ("az_trainer_set_comm", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    ("az_trainer_set_host_reducer", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    ("az_trainer_set_sharded", C.c_int, [C.c_void_p, C.c_int]),
    ("az_trainer_exchange_stats", C.c_int, [C.c_void_p, P(C.c_int64), P(C.c_int64), P(C.c_double), C.c_int]),
    ("az_trainer_time_exchanges", C.c_int, [C.c_void_p, C.c_int]),
    ("az_rules_probe", C.c_int, [C.c_int, P(AzPos), P(C.c_int32), C.c_int, P(AzPos), P(C.c_int32), P(C.c_int32),
                                 P(C.c_int32), P(C.c_int32), P(C.c_int32), P(C.c_int32), P(C.c_uint64), P(C.c_float)]),
]

if not os.path.exists(LIB_PATH):
    raise ImportError("libaz.so not built (%s); run __graft_entry__.build() or make -C %s" % (LIB_PATH, CSRC))

lib = C.CDLL(LIB_PATH)


def hip_runtime_paths():
    """HIP runtime(s) mapped in this process (libaz is built for /opt/rocm's; torch bundles
    another libamdhip64.so.7 with the same SONAME, so import azchess BEFORE torch)."""
    try:
        return sorted({l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l})
    except OSError:
        return []


_rt = hip_runtime_paths()
if _rt and not any(p.startswith("/opt/rocm") for p in _rt):
    import warnings
    warnings.warn("libaz bound to a non-/opt/rocm HIP runtime %s (torch imported first?)" % _rt)
for _name, _res, _args in SIGNATURES:
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


class AzError(RuntimeError):
    pass


def check(rc):
    if rc < 0:
        raise AzError(lib.az_last_error().decode())
    return rc


def fptr(a):
    return a.ctypes.data_as(P(C.c_float))


def i32ptr(a):
    return a.ctypes.data_as(P(C.c_int32))


def u32ptr(a):
    return a.ctypes.data_as(P(C.c_uint32))


def u64ptr(a):
    return a.ctypes.data_as(P(C.c_uint64))

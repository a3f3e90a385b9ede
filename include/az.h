/*
 * az.h -- C-ABI of the MI355X-native alphazero-chess self-play engine (libaz.so).
 *
 * Drop-in boundary for the reference's hot path (AlexandreGac/alphazero-chess @ 2025-08-24).
 * The reference is a single Rust crate with no FFI; each entry point below replaces one
 * item of its module surface (file:line cited) and is what a Rust `extern "C"` block
 * would bind (see INTEGRATION.md for the binding a maintainer would add).
 *
 * Conventions: every function returns int status (0 = ok, <0 = error; message via
 * az_last_error()) unless noted.  Plain pointers and sizes only.  Host buffers are
 * caller-owned; the engine owns all device memory.  A handle is used by one host thread
 * at a time (not re-entrant); one handle per GPU.
 * Squares: a1 = 0 ... h8 = 63 (shakmaty Square order).  Move indices: 0..4095 =
 * plane*64 + rank'*8 + file (chess.rs:73-116), rank' flipped for Black.
 */
#ifndef AZ_H
#define AZ_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AZ_ACTION_SPACE 4096   /* parameters.rs:3 */
#define AZ_PLANES 19           /* chess.rs:191-245 */
#define AZ_MAX_MOVES 256

/* Result codes of play (chess.rs:29-34 GameResult, plus -1 = Err("Illegal move")) */
enum { AZ_ONGOING = 0, AZ_DRAW = 1, AZ_WHITE_WINS = 2, AZ_BLACK_WINS = 3, AZ_ILLEGAL = -1 };

/* Packed position (80 bytes) -- the engine's replacement for shakmaty::Chess.
 * bb: P N B R Q K (both colours), white, black.  ep: pseudo-legal en-passant square
 * (shakmaty pseudo_legal_ep_square, chess.rs:218) or 64.  flags bit0: that ep capture is
 * also legal (shakmaty Chess equality uses the legal ep square).  castling bits:
 * 1 = White O-O, 2 = White O-O-O, 4 = Black O-O, 8 = Black O-O-O.
 * rep_key: hash of (board, turn, castling, legal ep) -- the repetition key. */
typedef struct az_pos {
    uint64_t bb[8];
    uint8_t turn, castling, ep, flags;
    uint16_t halfmoves, fullmoves;
    uint64_t rep_key;
} az_pos;

const char* az_last_error(void);
int az_version(void);
int az_device_count(int* n);
int az_device_synchronize(int device);                              /* hipDeviceSynchronize on `device` */

/* ---- rules & codec: chess.rs ---------------------------------------------------- */
int az_pos_startpos(az_pos* out);                                   /* Chess::new, chess.rs:21 */
int az_pos_from_fen(const char* fen, az_pos* out);
int az_pos_to_fen(const az_pos* p, char* buf, int cap);            /* Fen::from_position(.., PseudoLegal) */
uint64_t az_pos_fen_key(const az_pos* p);                           /* cache key, tree.rs:214 */
/* legal move indices in shakmaty legal_moves() order WITH duplicates for
 * under-promotions, exactly MCTree::new's `moves` (tree.rs:86-89). Returns count. */
int az_pos_legal_indices(const az_pos* p, int32_t* out, int cap);
/* index_to_move (chess.rs:118-171) + play_unchecked: returns 1 and writes the child
 * position if the index names a legal move, 0 otherwise. */
int az_pos_play_index(const az_pos* p, int32_t index, az_pos* child);
int az_move_to_index(int from, int to, int turn);                   /* chess.rs:73-116 */
/* outcome(): AZ_ONGOING, AZ_DRAW (stalemate / insufficient material), AZ_WHITE/BLACK_WINS */
int az_pos_outcome(const az_pos* p);
int az_pos_encode(const az_pos* p, float* out);                     /* to_tensor, chess.rs:191-245: 19*64 f32 */

/* GameState = position + repetition multiset (chess.rs:13-27) */
typedef struct az_game az_game;
int az_game_create(az_game** out);                                  /* GameState::new, chess.rs:20 */
int az_game_clone(const az_game* g, az_game** out);
int az_game_destroy(az_game* g);
int az_game_position(const az_game* g, az_pos* out);
int az_game_history(const az_game* g, int32_t* moves, int cap);     /* indices played so far; returns count */
/* play_move(state, index_to_move(index)) (chess.rs:36-63): AZ_ONGOING / AZ_DRAW /
 * AZ_WHITE_WINS / AZ_BLACK_WINS / AZ_ILLEGAL */
int az_game_play(az_game* g, int32_t index);

/* ---- network: agent.rs AlphaZero ------------------------------------------------- */
enum { AZ_DTYPE_F32 = 0, AZ_DTYPE_BF16 = 1 };
typedef struct { int blocks, filters, dtype; } az_net_desc;
typedef struct az_net az_net;
/* number of f32 parameters in the flat layout (see DESIGN.md "Weights"): burn module
 * order, conv [out,in,kh,kw], BatchNorm {gamma,beta,running_mean,running_var},
 * Linear weight [d_in,d_out] (burn layout). */
size_t az_net_num_params(int blocks, int filters);
/* AlphaZero::new + load_record (agent.rs:49-110, main.rs:109-116): weights copied to HBM,
 * BatchNorm folded into the convs (inference mode, model.valid()). */
int az_net_create(const az_net_desc* desc, const float* weights, size_t n, int device, az_net** out);
int az_net_destroy(az_net* net);
/* name of the kernel(s) that evaluate this net (fused f32 Winograd / f32 direct / bf16 / per-layer) */
int az_net_tower_kernel(az_net* net, char* out, int cap);
/* burn NamedMpkFileRecorder<FullPrecisionSettings> model files:
 * load_model (main.rs:109-116) -> flat weights for az_net_create / az_trainer_create, and
 * model.save_file (training.rs:269-270) from flat weights.  out/w hold az_net_num_params floats. */
int az_net_load_mpk(const char* path, int blocks, int filters, float* out, size_t n);
int az_net_save_mpk(const char* path, int blocks, int filters, const float* w, size_t n);
/* AlphaZero::forward (agent.rs:112-144): planes [n,19,8,8] f32 -> policy [n,4096]
 * (softmax) and value [n] (tanh). Host buffers. */
int az_net_forward(az_net* net, const float* planes, int n, float* policy, float* value);
/* Same on device pointers / a caller's hipStream_t (NULL = engine stream). */
int az_net_forward_device(az_net* net, const float* d_planes, int n, float* d_policy, float* d_value,
                          void* stream);

/* ---- search: tree.rs MCTree + training.rs self-play driver ------------------------ */
/* AZ_EVAL_NET: the engine's own az_net (fused HIP tower).  AZ_EVAL_SYNTHETIC: the hash evaluator
 * the oracle shares (parity tests).  AZ_EVAL_CALLBACK: a caller-owned evaluator installed with
 * az_search_set_evaluator -- the reference's InferenceRequest / process_batch boundary
 * (training.rs:28-31, 380-422; tree.rs:222-228), e.g. a Rust caller keeping its burn model. */
enum { AZ_EVAL_NET = 0, AZ_EVAL_SYNTHETIC = 1, AZ_EVAL_CALLBACK = 2 };
/* Caller-owned evaluator: called on the calling thread of az_search_set_roots / az_search_run /
 * az_selfplay_* once per simulation step with the n leaf positions that need an evaluation (every
 * game's pending InferenceRequest of that step, in batch-row order).  It fills policy[n * 4096]
 * (AlphaZero::forward's softmax row, agent.rs:128-130: the engine reads it at the legal move
 * indices only) and value[n] (side-to-move view, tanh output).  The rows must be what the
 * reference's forward gives: finite, non-negative, a softmax over the 4096 entries -- the engine
 * takes the legal entries as priors unchecked (PUCT of a NaN prior never wins a selection).
 * Return 0 on success; a non-zero return aborts the search call with an error.  Buffers are
 * engine-owned and valid for the call. */
typedef int (*az_eval_fn)(void* ctx, const az_pos* positions, int n, float* policy, float* value);
typedef struct {
    int games;          /* concurrent games G on this GPU (NUM_EPISODES, parameters.rs:13) */
    int sims;           /* simulations per move (NUM_SIMULATIONS, parameters.rs:32) */
    float c_puct;       /* parameters.rs:34 */
    float dir_alpha;    /* parameters.rs:28 */
    float dir_eps;      /* parameters.rs:29 */
    int temp_moves;     /* TEMPERATURE_ANNEALING, parameters.rs:31 */
    int noise;          /* Dirichlet noise at roots (training.rs:358, tree.rs:243) */
    uint64_t seed;      /* counter-based RNG seed (replaces thread_rng) */
    int evaluator;      /* AZ_EVAL_NET, AZ_EVAL_SYNTHETIC or AZ_EVAL_CALLBACK */
    int continuous;     /* self-play: restart a finished slot with a new game */
    int record_evals;   /* keep a log of every evaluation (for replay parity) */
    int eval_log_cap;   /* log capacity in rows */
    int cache_capacity; /* FEN evaluation cache entries (CACHE_CAPACITY, parameters.rs:4; 0 = off):
                           tree.rs:214-219 lookup, training.rs:413 insert.  Changes only how many
                           network rows run, never a result. */
} az_search_cfg;
typedef struct az_search az_search;

int az_search_default_cfg(az_search_cfg* cfg);   /* reference defaults (parameters.rs) */
int az_search_create(az_net* net, const az_search_cfg* cfg, int device, az_search** out);
int az_search_destroy(az_search* s);
/* Install the AZ_EVAL_CALLBACK evaluator (cfg.evaluator must be AZ_EVAL_CALLBACK); replaces
 * process_batch (training.rs:380-422).  Must precede the first az_search_set_roots /
 * az_selfplay_reset. */
int az_search_set_evaluator(az_search* s, az_eval_fn fn, void* ctx);

/* Roots from histories: game g's root = startpos + hist[off[g]..off[g+1]) (move indices),
 * evaluated and optionally noised: MCTree::new(policy, state, apply_noise), tree.rs:84-104.
 * noise_ply[g] (may be NULL = 0) selects the RNG stream (seed, game_id[g], ply).  Abandons a
 * self-play move left in progress by az_selfplay_run_sims (its simulations are discarded). */
int az_search_set_roots(az_search* s, const int32_t* hist, const int32_t* off, const int32_t* game_id,
                        const int32_t* noise_ply, int apply_noise);
/* The same from arbitrary states, MCTree::new(policy, state, apply_noise) with any GameState
 * (tree.rs:84-104): game g's state starts at start[g] (NULL = startpos for every game; its
 * repetition multiset holds start[g] once) and plays hist[off[g]..off[g+1]) through play_move, so
 * the root is the last position and every earlier one counts toward threefold (chess.rs:52-60). */
int az_search_set_roots_from(az_search* s, const az_pos* start, const int32_t* hist, const int32_t* off,
                             const int32_t* game_id, const int32_t* noise_ply, int apply_noise);
/* monte_carlo_tree_search for every game (tree.rs:106-115 / 169-178).  Outputs (any may
 * be NULL): improved policy [G,4096], visits [G,4096], max_subtree_depth [G]. */
int az_search_run(az_search* s, float* improved, uint32_t* visits, int32_t* depth);
/* The current roots' visits / improved policy / max_subtree_depth without running simulations:
 * the reference's public MCTree fields (tree.rs:25-34), e.g. mid-move during az_selfplay_run_sims. */
int az_search_read_roots(az_search* s, float* improved, uint32_t* visits, int32_t* depth);
/* traverse_new(action, apply_noise) for every game (tree.rs:239-256) after playing the
 * action on its GameState (training.rs:323-325).  result[g] receives the play_move result. */
int az_search_advance(az_search* s, const int32_t* actions, int apply_noise, int32_t* result);

/* run_all_episodes (training.rs:340-378): reset all G slots to new games from startpos */
int az_selfplay_reset(az_search* s);
/* one move for every active game: sims, improved policy, action choice (training.rs:310-321),
 * play, traverse/record.  *finished = games that ended in this step. */
int az_selfplay_step(az_search* s, int* finished, int* active);
/* The same move in pieces: the next `nsims` simulation steps of every game's current move
 * (async_monte_carlo_tree_search's loop, tree.rs:169-178, cut at any simulation boundary).
 * When the move's sims are complete (*move_done = 1) the action choice, play and re-root of
 * az_selfplay_step follow; until then *finished = 0, *active = -1.  Results are identical to
 * az_selfplay_step. */
int az_selfplay_run_sims(az_search* s, int nsims, int* finished, int* active, int* move_done);

/* EpisodeStep (training.rs:15-20) of finished games, drained in game order. */
typedef struct {
    int32_t game_id;
    int32_t ply;
    int32_t action;
    int32_t search_depth;
    float final_value;         /* training.rs:332-335 */
    int32_t result;            /* AZ_DRAW / AZ_WHITE_WINS / AZ_BLACK_WINS */
    int32_t nvis;              /* improved_policy = visits / sum(visits) over these entries */
    az_pos state;
    uint16_t vis_idx[224];
    uint16_t vis_n[224];
} az_episode_step;
int az_selfplay_drain(az_search* s, az_episode_step* out, int cap);   /* returns count */

typedef struct {
    int64_t sims;              /* simulations completed */
    int64_t evals;             /* network rows evaluated */
    int64_t terminal_leaves;
    int64_t games_finished;
    int64_t moves;
    int64_t max_depth_sum;     /* sum over moves of max_subtree_depth */
    int64_t cache_hits;        /* expansions served by the FEN cache (CACHE_HITS, training.rs:12) */
    int64_t cache_misses;      /* expansions that needed a network row (CACHE_MISSES) */
    int64_t overflow;          /* expansions refused for want of node/edge arena space (0 by construction) */
    int64_t max_nodes;         /* largest node count of any game's current tree (arena: sims + 2) */
    int64_t max_edges;         /* largest edge count of any game's current tree */
    int64_t node_cap, edge_cap;/* the per-game arena sizes */
} az_search_stats;
int az_search_stats_get(az_search* s, az_search_stats* out);
/* 1 if the untimed simulation steps run through the persistent per-game kernel (k_sims32w: a
 * game's backup / select / expand and its Winograd f32 evaluation in one workgroup, no grid-wide
 * step boundary; chosen when the games fit the device in one round, the net is f32 Winograd (or the
 * bf16 64-filter tower) and
 * the FEN cache is off; env AZ_PERSIST=0/1 forces it), 0 if they run as k_step + the batched
 * tower.  Either way the results are identical (tests/test_gpu_search.py). */
int az_search_persistent(az_search* s);

/* Evaluation log (cfg.record_evals): keys[n] (fen keys), values[n], CSR priors at the
 * legal move indices. Pass NULL arrays to query sizes. */
int az_search_eval_log(az_search* s, int64_t* n_rows, int64_t* n_priors, uint64_t* keys, float* values,
                       int32_t* off, int32_t* idx, float* priors);

/* Profiling: device times measured with HIP events on the engine stream while enabled, on
 * every 32nd simulation step (steps 0, 32, 64, ...; every field except select_bytes covers
 * those sampled steps only: sim_steps = sampled steps = select_launches).
 * conv_*: the first residual 3x3 FxF conv of every simulation step (the dominant kernel);
 * conv_flop = algorithmic FLOPs of those launches (rows * 2*64*9*F*F).  tower_*: the whole
 * conv tower.  select_bytes: algorithmic bytes read by the select walk (16 B per edge +
 * 16 B node + 4 B sqrt per level). */
typedef struct {
    double conv_ms;      int64_t conv_launches;  double conv_flop;
    double tower_ms;     double tower_flop;
    double select_ms;    int64_t select_launches; double select_bytes;
    double expand_ms;    double encode_ms;       double heads_ms;    double backup_ms;
    double sim_step_ms;  int64_t sim_steps;      int64_t rows;
} az_timing;
int az_search_timing(az_search* s, az_timing* out, int reset, int enable);


/* ---- training: training.rs train() inner loop ---------------------
 * f32 end to end (the reference's precision).  The trainer owns a device copy of the flat
 * parameters (az_net_num_params layout, BatchNorm running statistics included), the AdamW
 * moments and every activation of a batch of up to max_batch positions. */
typedef struct az_trainer az_trainer;
/* get_cyclical_lr (training.rs:424-441) */
double az_cyclical_lr(int iteration);
/* AlphaZero::new/load_record + AdamWConfig::new().with_grad_clipping(Value(1.0))
 * .with_weight_decay(1e-4).init() (training.rs:48-66) */
int az_trainer_create(int blocks, int filters, const float* weights, size_t n, int max_batch, int device,
                      az_trainer** out);
int az_trainer_destroy(az_trainer* t);
/* forward (training-mode BatchNorm, running statistics updated) + compute_gradients
 * (training.rs:277-292) for one batch: planes [B,19,8,8] (to_tensor), target policy [B,4096],
 * target value [B].  losses (may be NULL) = {policy_loss, value_loss} batch means. */
int az_trainer_compute_grads(az_trainer* t, const float* planes, const float* target_policy,
                             const float* target_value, int batch, float* losses);
/* gradient all-reduce over the trainer's communicator (if any), clip by value 1.0,
 * AdamW step with learning rate lr (optimizer.step, training.rs:186-189) */
int az_trainer_apply(az_trainer* t, double lr);
/* compute_grads + apply: one iteration of training.rs:147-190 */
int az_trainer_step(az_trainer* t, const float* planes, const float* target_policy, const float* target_value,
                    int batch, double lr, float* losses);
/* flat parameters (to build an az_net for self-play, or to save) / last gradients */
int az_trainer_get_params(az_trainer* t, float* out, size_t n);
int az_trainer_get_grads(az_trainer* t, float* out, size_t n);
/* introspection for parity tests: the activation each ReLU of the last forward acted on, in
 * forward order -- layer 0 = input block output, 1..2B = residual blocks (h_b, x_b+1 NHWC
 * [B*64][F]), 2B+1 = head convs after BN+ReLU [B*64][64] (columns 0..39), 2B+2 =
 * value_linear_1 output before its ReLU [B][64].  n must equal the tensor's size. */
int az_trainer_relu_output(az_trainer* t, int layer, float* out, size_t n);
/* device time (HIP events on the trainer stream) summed over steps: whole step (compute_grads
 * start to apply end) and the gradient all-reduce; reset = zero the sums after reading */
int az_trainer_timing(az_trainer* t, double* step_ms, double* allreduce_ms, int64_t* steps, int reset);
/* data-parallel training over RCCL (xGMI): rank 0 creates the id (128 bytes, returns its
 * size), every rank passes it to az_trainer_set_comm. */
int az_comm_unique_id(void* out, int cap);
int az_trainer_set_comm(az_trainer* t, const void* unique_id, int rank, int world);
/* The same data-parallel step with the exchange done by the caller on the host (no RCCL: e.g.
 * gloo / MPI between hosts, or a test driving two ranks in one process): at each apply, fn(ctx,
 * buf, n) must replace buf[0..n) (host memory) by its element-wise sum over the `world` ranks --
 * once for the gradients (before clipping; the AdamW step then scales by 1/world) and once for
 * the BatchNorm running statistics (then scaled by 1/world).  Return 0 on success.  Replaces a
 * communicator set by az_trainer_set_comm. */
typedef int (*az_allreduce_fn)(void* ctx, float* buf, size_t n);
int az_trainer_set_host_reducer(az_trainer* t, az_allreduce_fn fn, void* ctx, int rank, int world);
/* Sharded batch (on = 1): each rank's az_trainer_compute_grads batch is its shard of ONE global
 * batch -- the reference's single BATCH_SIZE = 512 step (training.rs:137-159, parameters.rs:17)
 * split over the ranks.  Every training-mode BatchNorm normalises with the statistics of the whole
 * global batch (agent.rs:37,41,115,125,134): each BN's per-rank (sum, squared deviations, rows)
 * are exchanged in the forward and its (sum dz, sum dz*yhat) in the backward, through the
 * communicator or host reducer (a sum all-reduce each: 2 per BatchNorm per step, 43 BNs at
 * 20x256); the loss and the BN backward normalise by the global row count, the summed gradient is
 * applied unscaled, the running statistics (identical on every rank) are not averaged, and the
 * reported losses are global means.  Off (default): each rank trains its own batch with per-rank
 * BatchNorm statistics and the gradients are averaged (global batch = batch x world).  At one rank
 * both modes compute the same step bit for bit. */
int az_trainer_set_sharded(az_trainer* t, int on);
/* the exchanges of the data-parallel steps since the last reset (RCCL all-reduces or host
 * reductions: sharded BatchNorm statistics and backward sums, losses, gradients, running
 * statistics): how many, over how many applied steps, and -- while az_trainer_time_exchanges(t, 1)
 * is on (off by default: the events cost queue time) -- their device time (HIP events around each
 * one on the trainer stream) */
int az_trainer_exchange_stats(az_trainer* t, int64_t* collectives, int64_t* steps, double* exchange_ms, int reset);
int az_trainer_time_exchanges(az_trainer* t, int on);

/* ---- replay buffer: memory.rs ReplayBuffer, host memory ------------ */
typedef struct az_replay az_replay;
int az_replay_create(int capacity, az_replay** out);                /* ReplayBuffer::new, memory.rs:33-38 */
int az_replay_destroy(az_replay* r);
int az_replay_len(const az_replay* r);                              /* memory.rs:103-105 */
/* ReplayBuffer::add (memory.rs:41-79): running mean into an existing FEN entry (returns 0) or
 * a new entry at the FIFO's end, evicting the oldest at capacity (returns 1) */
int az_replay_add(az_replay* r, const az_episode_step* step);
/* az_replay_add of steps[0..n) in order; returns the number of new unique positions (the union of
 * every rank's drained steps, added in rank order, keeps the replicas of one buffer identical) */
int az_replay_add_many(az_replay* r, const az_episode_step* steps, int n);
int az_replay_add_dense(az_replay* r, const az_pos* state, const float* policy, float value);
/* ReplayBuffer::sample (memory.rs:81-101): min(batch, len) distinct entries, uniformly (seeded);
 * writes to_tensor planes [n,19,64], policies [n,4096], values [n], positions (any may be NULL).
 * Returns n. */
int az_replay_sample(az_replay* r, int batch, uint64_t seed, float* planes, float* policy, float* value,
                     az_pos* states);
/* save / load (memory.rs:107-117): bincode 2 standard-config file of the reference's layout */
int az_replay_save(const az_replay* r, const char* path);
int az_replay_load(const char* path, int capacity, az_replay** out);

/* ---- test hook: the device rules path (parity tests; the engine never calls it) ----------
 * Runs, on the GPU, exactly what a leaf expansion runs (index_to_move + play, chess.rs:118-171 /
 * 42; the wave-parallel legal move generator; outcome(), chess.rs:43-50; the legal-ep flag and
 * repetition key) plus the roots' serial generator and the towers' plane staging (to_tensor,
 * chess.rs:191-245), for n items: item i = parent[i] with action[i] played (action[i] < 0: parent[i]
 * itself; an illegal action is refused on the host).  Outputs (child required, the rest may be NULL):
 * child[n] (flags, rep_key set); moves[n][256] / nmoves[n]: the leaf generator's legal indices in
 * shakmaty order with under-promotion duplicates (MCTree::new's `moves`, tree.rs:86-89);
 * root_moves[n][256] / root_n[n]: the same from the roots' generator; outcome[n] (AZ_ONGOING /
 * AZ_DRAW / AZ_WHITE_WINS / AZ_BLACK_WINS, no repetition); in_check[n]; fen_key[n] (the FEN-cache
 * key, tree.rs:214); planes[n][19][64]. */
int az_rules_probe(int device, const az_pos* parent, const int32_t* action, int n, az_pos* child, int32_t* moves,
                   int32_t* nmoves, int32_t* root_moves, int32_t* root_n, int32_t* outcome, int32_t* in_check,
                   uint64_t* fen_key, float* planes);

#ifdef __cplusplus
}
#endif
#endif

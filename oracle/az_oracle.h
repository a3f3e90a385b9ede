/*
 * az_oracle.h -- CPU ORACLE for the alphazero-chess self-play hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (alphazero-chess_amd/) links,
 * imports or calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, always as the checker / CPU baseline, never as the
 * thing measured or shipped.
 *
 * It is a plain-C restatement of the reference's algorithm (AlexandreGac/alphazero-chess
 * @ 2025-08-24, Rust): every function cites the reference file:line it follows.
 * The reference itself cannot be built here (no cargo/rustc, crates not vendored),
 * and it has no tests or golden vectors, so parity is pinned by:
 *   - canonical perft counts (move generator), see tests/test_oracle_chess.py,
 *   - fixed move-index tables,
 *   - torch-CPU golden vectors for the network (tests/golden/, script committed),
 *   - the reference's third-party semantics (shakmaty 0.29.0 move order / outcome /
 *     repetition equality, rand_distr 0.4.3 Gamma/Dirichlet) restated from their
 *     published algorithms.  Where those are recalled rather than checkable here the
 *     result is "parity unpinned" for that aspect (DESIGN.md, section Oracle).
 *
 * Representation here is deliberately different from the product's (mailbox board,
 * make-and-test legality, sort into shakmaty order) so the two are independent.
 */
#ifndef AZ_ORACLE_H
#define AZ_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define REF_ACTION_SPACE 4096          /* parameters.rs:3 */
#define REF_NUM_HALFMOVES 100          /* chess.rs:9 */
#define REF_NUM_FULLMOVES 200          /* chess.rs:10 */
#define REF_REPETITIONS 3              /* chess.rs:11 */
#define REF_MAX_MOVES 256

/* piece codes: +1..+6 white P N B R Q K, -1..-6 black */
typedef struct {
    int8_t sq[64];      /* a1 = 0, h1 = 7, a8 = 56 (shakmaty Square order) */
    int32_t turn;       /* 0 white, 1 black */
    int32_t castling;   /* bit0 W O-O, bit1 W O-O-O, bit2 B O-O, bit3 B O-O-O */
    int32_t ep;         /* square skipped by the last double push, or -1 */
    int32_t halfmoves;
    int32_t fullmoves;
} ref_pos;

/* kind: 0 normal, 1 en passant, 2 castle (to = rook square, shakmaty Move::to()) */
typedef struct { int16_t from, to; int8_t promo; int8_t kind; } ref_move;

enum { REF_ONGOING = 0, REF_DRAW = 1, REF_WHITE_WINS = 2, REF_BLACK_WINS = 3, REF_ILLEGAL = -1 };

/* ---- chess rules (chess.rs + shakmaty semantics) ---- */
void ref_startpos(ref_pos* p);
int  ref_from_fen(const char* fen, ref_pos* p);          /* 0 ok */
int  ref_to_fen(const ref_pos* p, char* out, int cap);   /* FEN with pseudo-legal ep */
int  ref_legal_moves(const ref_pos* p, ref_move* out);   /* shakmaty legal_moves() order */
int  ref_in_check(const ref_pos* p);
int  ref_pseudo_legal_ep(const ref_pos* p);              /* -1 if none */
int  ref_legal_ep(const ref_pos* p);
int  ref_insufficient_material(const ref_pos* p);
void ref_play_unchecked(ref_pos* p, ref_move m);
int  ref_outcome(const ref_pos* p);                      /* REF_ONGOING if unknown */
uint64_t ref_perft(const ref_pos* p, int depth);
int  ref_move_to_index(ref_move m, int turn);            /* chess.rs:73-116 */
int  ref_index_to_move(int index, const ref_pos* p, ref_move* out); /* chess.rs:118-171; 1 if Some */
void ref_to_tensor(const ref_pos* p, float* out);        /* chess.rs:191-245, 19*64 */
int  ref_legal_indices(const ref_pos* p, int32_t* out);  /* tree.rs:86-89 (with duplicates) */
uint64_t ref_fen_key(const ref_pos* p);                  /* hash of FEN(PseudoLegal) content */
void ref_pos_bitboards(const ref_pos* p, uint64_t* bb8); /* P N B R Q K white black */

/* GameState: position + repetition multiset (chess.rs:13-27) */
typedef struct {
    ref_pos position;
    int32_t n;          /* number of (key,count) entries */
    int32_t cap;
    ref_pos* keys;      /* stored positions (compared with shakmaty Chess equality) */
    int32_t* counts;
} ref_game;
void ref_game_new(ref_game* g);                           /* chess.rs:20-26 */
void ref_game_from(ref_game* g, const ref_pos* start);      /* repetition multiset {start: 1} */
void ref_game_clone(ref_game* dst, const ref_game* src);
void ref_game_free(ref_game* g);
int  ref_play_move(ref_game* g, ref_move m);              /* chess.rs:36-63 */
int  ref_chess_eq(const ref_pos* a, const ref_pos* b);    /* shakmaty Chess PartialEq */

/* ---- deterministic counter-based RNG + arithmetic (replaces thread_rng) ---- */
uint64_t ref_splitmix64(uint64_t x);
uint64_t ref_stream_key(uint64_t seed, uint64_t game, uint64_t ply, uint64_t purpose);
float ref_open01(uint64_t key, uint64_t* ctr);
float ref_uniform01(uint64_t key, uint64_t* ctr);
float ref_det_logf(float x);
float ref_det_expf(float x);
float ref_gamma(float shape, uint64_t key);               /* rand_distr 0.4.3 Gamma(shape,1) */
void  ref_dirichlet(float alpha, int n, uint64_t key, float* out); /* rand_distr Dirichlet */

/* ---- network (agent.rs) fp32, BN applied as in burn inference mode ---- */
size_t ref_net_num_params(int blocks, int filters);
typedef struct ref_net ref_net;
ref_net* ref_net_create(int blocks, int filters, const float* flat);
void ref_net_free(ref_net* n);
void ref_net_forward(const ref_net* n, const float* planes, int batch, float* policy, float* value, int threads);

/* ---- MCTS (tree.rs) + self-play driver (training.rs) ---- */
typedef struct {
    int sims;            /* NUM_SIMULATIONS parameters.rs:32 */
    float c_puct;        /* parameters.rs:34 */
    float dir_alpha;     /* parameters.rs:28 */
    float dir_eps;       /* parameters.rs:29 */
    int temp_moves;      /* TEMPERATURE_ANNEALING parameters.rs:31 */
    int noise;           /* apply Dirichlet at roots (training.rs:358) */
    uint64_t seed;
    int eval_kind;       /* 0 synthetic hash evaluator, 1 net, 2 replay table */
    const ref_net* net;
    int threads;
} ref_search_cfg;

/* replay table: evaluations recorded by the GPU, keyed by fen key */
typedef struct ref_replay ref_replay;
ref_replay* ref_replay_create(int64_t n, const uint64_t* keys, const float* values,
                              const int32_t* prior_off, const float* priors, const int32_t* prior_idx);
void ref_replay_free(ref_replay* r);

/* Synthetic deterministic evaluator, shared definition with the GPU path. */
void ref_synth_eval(const ref_pos* p, float* dense_policy, float* value);

/* One search from a GameState. Outputs root visits[4096] (f32 as the reference),
 * improved policy[4096], max_subtree_depth, NN-eval count. */
typedef struct {
    float visits[REF_ACTION_SPACE];
    float improved[REF_ACTION_SPACE];
    int depth;
    int64_t evals;
} ref_search_out;

/* Self-play of ngames games, lockstep batched like run_all_episodes (training.rs:340-378).
 * Writes per-step records; returns number of steps written (<= cap). */
typedef struct {
    int32_t game, ply;
    int32_t action;          /* chosen index */
    int32_t depth;           /* max_subtree_depth */
    float final_value;       /* training.rs:332-335 */
    int32_t result;          /* game result code */
    uint64_t fen_key;
    int32_t nvis;            /* number of nonzero root visit entries */
    int32_t vis_idx[256];
    float vis_n[256];
} ref_step;

/* Search from startpos + a history of move indices (play_move each), as
 * MCTree::new(eval(root), state, noise) + monte_carlo_tree_search. 0 ok. */
int ref_search_game(const ref_search_cfg* cfg, const ref_replay* rep, const int32_t* history, int nhist,
                    int noise, uint64_t noise_key, ref_search_out* out);

/* The same from an arbitrary position: GameState{start, {start: 1}} + history (tree.rs:84-104). */
int ref_search_from(const ref_search_cfg* cfg, const ref_replay* rep, const ref_pos* start, const int32_t* history,
                    int nhist, int noise, uint64_t noise_key, ref_search_out* out);

/* rules parity test data: packed positions, and the rules answers for (parent, index) items */
void ref_pack(const ref_pos* p, int64_t n, uint64_t* bb, int32_t* meta);
int64_t ref_rules_batch(const ref_pos* parent, const int32_t* action, int64_t n, ref_pos* child, int32_t* moves,
                        int32_t* nmoves, int32_t* outcome, int32_t* in_check, int32_t* legal_ep, uint64_t* fen_key,
                        float* planes);
/* rules parity test data: uniform random playouts from the startpos, (parent, index) per ply */
int64_t ref_random_playouts(uint64_t seed, int ngames, int max_plies, ref_pos* parents, int32_t* actions,
                            int64_t cap);

int64_t ref_selfplay(const ref_search_cfg* cfg, const ref_replay* rep, int ngames, int max_plies,
                     ref_step* steps, int64_t cap, int64_t* sims_done, int64_t* evals_done);

/* The same self-play in lockstep with ONE batched evaluation per simulation step over every game's
 * pending leaf (the reference's batcher, training.rs:369-422; the CPU baseline of SURVEY 8d):
 * fn(ctx, planes [n][19][64] (to_tensor), n, policy [n][4096] out, value [n] out) -> 0 ok.
 * fn == NULL: cfg->eval_kind per row.  Same records as ref_selfplay. */
typedef int (*ref_eval_batch_fn)(void* ctx, const float* planes, int n, float* policy, float* value);
int64_t ref_selfplay_batched(const ref_search_cfg* cfg, int ngames, int max_plies, ref_eval_batch_fn fn, void* ctx,
                             ref_step* steps, int64_t cap, int64_t* sims_done, int64_t* evals_done);

/* ---- arena / Elo (validation.rs:284-384, ratings.rs:113-144) ---- */
int  ref_arena_choose(const float* policy, int fullmoves, int num_stochastic_moves, float u);
void ref_mask_to_legal(const ref_pos* p, float* policy);
void ref_compute_elos(const float* wm, int n, float base_elo, float* elos);   /* n <= 64 */

#ifdef __cplusplus
}
#endif
#endif

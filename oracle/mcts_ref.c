/*
 * mcts_ref.c -- ORACLE (test infrastructure only, see az_oracle.h).
 *
 * Faithful restatement of the reference search and self-play driver, keeping its
 * data structure (dense 4096-wide policy/visits/scores per node, child map, a
 * cloned GameState per node) and its float operation order:
 *   tree.rs:84-104   MCTree::new (legal index list with duplicates, optional noise)
 *   tree.rs:106-115  monte_carlo_tree_search + improved policy visits^(1/T)/sum
 *   tree.rs:117-144  simulation: Nt = sum(visits)+1, u = C*P*sqrt(Nt)/(1+N),
 *                    q = N>0 ? W/N : 0, strict '>' argmax (first max), backup
 *   tree.rs:146-167  expand: clone state, index_to_move, play_move, evaluate
 *   tree.rs:239-256  traverse_new (keep child moves/state/policy, re-noise, reset)
 *   tree.rs:258-269  max_subtree_depth
 *   tree.rs:272-289  apply_dirichlet_noise
 *   training.rs:294-338 run_episode (argmax with LAST max at fullmoves>=15, else
 *                    WeightedIndex sampling; final value turn*result*(1-fm/400))
 * Evaluations are pure functions of the position, so games are independent and the
 * reference's cross-game batching (training.rs:340-422) cannot change any result;
 * the oracle therefore runs games in parallel threads with batch-1 evaluations.
 */
#include "az_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

/* ---------------- evaluators ---------------- */

struct ref_replay {
    int64_t n, cap;          /* open-addressing table */
    uint64_t* keys;
    int64_t* slot;           /* row index or -1 */
    const float* values;
    const int32_t* off;
    const float* priors;
    const int32_t* idx;
};

ref_replay* ref_replay_create(int64_t n, const uint64_t* keys, const float* values,
                              const int32_t* prior_off, const float* priors, const int32_t* prior_idx) {
    ref_replay* r = (ref_replay*)calloc(1, sizeof(ref_replay));
    int64_t cap = 16;
    while (cap < 2 * n + 16) cap *= 2;
    r->cap = cap; r->n = n;
    r->keys = (uint64_t*)calloc((size_t)cap, sizeof(uint64_t));
    r->slot = (int64_t*)malloc((size_t)cap * sizeof(int64_t));
    for (int64_t i = 0; i < cap; i++) r->slot[i] = -1;
    r->values = values; r->off = prior_off; r->priors = priors; r->idx = prior_idx;
    for (int64_t i = 0; i < n; i++) {
        uint64_t h = keys[i] & (uint64_t)(cap - 1);
        while (r->slot[h] >= 0 && r->keys[h] != keys[i]) h = (h + 1) & (uint64_t)(cap - 1);
        if (r->slot[h] < 0) { r->keys[h] = keys[i]; r->slot[h] = i; }
    }
    return r;
}

void ref_replay_free(ref_replay* r) {
    if (!r) return;
    free(r->keys); free(r->slot); free(r);
}

static int replay_eval(const ref_replay* r, const ref_pos* p, float* policy, float* value) {
    uint64_t key = ref_fen_key(p);
    uint64_t h = key & (uint64_t)(r->cap - 1);
    while (r->slot[h] >= 0 && r->keys[h] != key) h = (h + 1) & (uint64_t)(r->cap - 1);
    if (r->slot[h] < 0) return -1;
    int64_t row = r->slot[h];
    memset(policy, 0, sizeof(float) * REF_ACTION_SPACE);
    for (int32_t j = r->off[row]; j < r->off[row + 1]; j++) policy[r->idx[j]] = r->priors[j];
    *value = r->values[row];
    return 0;
}

/* Synthetic evaluator: priors over the distinct legal indices from a
 * SplitMix64 of the FEN key, P = w / sum(w) with integer weights (exact), value in
 * [-1,1] on a 1e-3 grid.  The product implements the same definition on device. */
void ref_synth_eval(const ref_pos* p, float* policy, float* value) {
    uint64_t key = ref_fen_key(p);
    int32_t idx[REF_MAX_MOVES];
    int n = ref_legal_indices(p, idx);
    uint32_t w[REF_MAX_MOVES];
    uint32_t total = 0;
    memset(policy, 0, sizeof(float) * REF_ACTION_SPACE);
    for (int i = 0; i < n; i++) {
        int dup = 0;
        for (int j = 0; j < i; j++) if (idx[j] == idx[i]) dup = 1;
        w[i] = dup ? 0u : 1u + (uint32_t)(ref_splitmix64(key ^ ((uint64_t)(idx[i] + 1) * 0x9E3779B97F4A7C15ULL)) >> 48);
        total += w[i];
    }
    for (int i = 0; i < n; i++) if (w[i]) policy[idx[i]] = (float)w[i] / (float)total;
    int64_t v = (int64_t)(ref_splitmix64(key ^ 0x5BD1E9955BD1E995ULL) % 2001ULL) - 1000;
    *value = (float)v / 1000.0f;
}

typedef struct {
    const ref_search_cfg* cfg;
    const ref_replay* rep;
    int64_t evals;
    int failed;
} eval_ctx;

static void evaluate(eval_ctx* ctx, const ref_pos* p, float* policy, float* value) {
    ctx->evals++;
    if (ctx->cfg->eval_kind == 0) { ref_synth_eval(p, policy, value); return; }
    if (ctx->cfg->eval_kind == 2) {
        if (replay_eval(ctx->rep, p, policy, value) != 0) {
            ctx->failed = 1;
            memset(policy, 0, sizeof(float) * REF_ACTION_SPACE);
            *value = 0.0f;
        }
        return;
    }
    float planes[19 * 64];
    ref_to_tensor(p, planes);
    ref_net_forward(ctx->cfg->net, planes, 1, policy, value, 1);
}

/* ---------------- MCTree ---------------- */

typedef struct mct {
    int nchild, capchild;
    int32_t* child_idx;
    struct mct** child;
    int nmoves;
    int32_t moves[REF_MAX_MOVES];
    ref_game state;
    float* policy;
    float* visits;
    float* scores;
} mct;

static void apply_dirichlet_noise(const ref_search_cfg* cfg, float* policy, const int32_t* moves, int n,
                                  uint64_t key) {
    if (n < 2) return;                                             /* tree.rs:273-275 */
    float eta[REF_MAX_MOVES];
    ref_dirichlet(cfg->dir_alpha, n, key, eta);                    /* tree.rs:277-280 */
    float keep = 1.0f - cfg->dir_eps;
    for (int i = 0; i < REF_ACTION_SPACE; i++) policy[i] *= keep; /* tree.rs:282-284 */
    for (int k = 0; k < n; k++) policy[moves[k]] += cfg->dir_eps * eta[k]; /* tree.rs:286-288 */
}

static mct* mct_new(const ref_search_cfg* cfg, const float* policy, const ref_game* state, int noise,
                    uint64_t noise_key) {
    mct* t = (mct*)calloc(1, sizeof(mct));
    ref_game_clone(&t->state, state);
    t->nmoves = ref_legal_indices(&t->state.position, t->moves);
    t->policy = (float*)malloc(sizeof(float) * REF_ACTION_SPACE);
    t->visits = (float*)calloc(REF_ACTION_SPACE, sizeof(float));
    t->scores = (float*)calloc(REF_ACTION_SPACE, sizeof(float));
    memcpy(t->policy, policy, sizeof(float) * REF_ACTION_SPACE);
    if (noise) apply_dirichlet_noise(cfg, t->policy, t->moves, t->nmoves, noise_key);
    return t;
}

static void mct_free(mct* t) {
    if (!t) return;
    for (int i = 0; i < t->nchild; i++) mct_free(t->child[i]);
    free(t->child_idx); free(t->child);
    ref_game_free(&t->state);
    free(t->policy); free(t->visits); free(t->scores);
    free(t);
}

static mct* mct_find(mct* t, int idx) {
    for (int i = 0; i < t->nchild; i++) if (t->child_idx[i] == idx) return t->child[i];
    return NULL;
}

static void mct_insert(mct* t, int idx, mct* c) {
    if (t->nchild == t->capchild) {
        t->capchild = t->capchild ? t->capchild * 2 : 4;
        t->child_idx = (int32_t*)realloc(t->child_idx, sizeof(int32_t) * (size_t)t->capchild);
        t->child = (mct**)realloc(t->child, sizeof(mct*) * (size_t)t->capchild);
    }
    t->child_idx[t->nchild] = idx;
    t->child[t->nchild] = c;
    t->nchild++;
}

static float mct_expand(mct* t, eval_ctx* ctx, int max_index) {
    ref_game leaf;
    ref_game_clone(&leaf, &t->state);                              /* tree.rs:147 */
    ref_move m;
    if (!ref_index_to_move(max_index, &leaf.position, &m)) {       /* tree.rs:148 */
        fprintf(stderr, "oracle: Illegal move! %d\n", max_index);
        abort();
    }
    int r = ref_play_move(&leaf, m);                               /* tree.rs:149 */
    float value;
    if (r == REF_ONGOING) {
        float* policy = (float*)malloc(sizeof(float) * REF_ACTION_SPACE);
        evaluate(ctx, &leaf.position, policy, &value);             /* tree.rs:151-158 */
        mct_insert(t, max_index, mct_new(ctx->cfg, policy, &leaf, 0, 0)); /* tree.rs:159 */
        free(policy);
    } else if (r == REF_DRAW) {
        value = 0.0f;                                              /* tree.rs:163 */
    } else if (r == REF_ILLEGAL) {
        fprintf(stderr, "oracle: illegal move picked %d\n", max_index);
        abort();
    } else {
        value = -1.0f;                                             /* tree.rs:164 */
    }
    ref_game_free(&leaf);
    return value;
}

static float mct_simulation(mct* t, eval_ctx* ctx) {
    float max_value = -INFINITY;
    int max_index = 0;
    float total_visits = 0.0f;
    for (int i = 0; i < REF_ACTION_SPACE; i++) total_visits += t->visits[i];
    total_visits = total_visits + 1.0f;                            /* tree.rs:121 */
    float c = ctx->cfg->c_puct;
    for (int k = 0; k < t->nmoves; k++) {                          /* tree.rs:123-132 */
        int i = t->moves[k];
        float u_value = c * t->policy[i] * sqrtf(total_visits) / (1.0f + t->visits[i]);
        float q_value = t->visits[i] > 0.0f ? t->scores[i] / t->visits[i] : 0.0f;
        float value = q_value + u_value;
        if (value > max_value) { max_value = value; max_index = i; }
    }
    mct* node = mct_find(t, max_index);
    float value = node ? -mct_simulation(node, ctx) : -mct_expand(t, ctx, max_index);
    t->scores[max_index] += value;                                 /* tree.rs:141-142 */
    t->visits[max_index] += 1.0f;
    return value;
}

static int mct_depth(const mct* t) {
    int best = -1;
    for (int i = 0; i < t->nchild; i++) {
        int d = mct_depth(t->child[i]);
        if (d > best) best = d;
    }
    return best < 0 ? 0 : 1 + best;
}

static void mct_search(mct* t, eval_ctx* ctx, ref_search_out* out) {
    for (int s = 0; s < ctx->cfg->sims; s++) mct_simulation(t, ctx);
    float sum = 0.0f;
    for (int i = 0; i < REF_ACTION_SPACE; i++) sum += t->visits[i];  /* T = 1: powf(n, 1) = n */
    for (int i = 0; i < REF_ACTION_SPACE; i++) {
        out->visits[i] = t->visits[i];
        out->improved[i] = t->visits[i] / sum;
    }
    out->depth = mct_depth(t);
}

static mct* mct_traverse_new(mct* t, int action, const ref_search_cfg* cfg, int noise, uint64_t key) {
    mct* c = NULL;
    for (int i = 0; i < t->nchild; i++) {
        if (t->child_idx[i] == action) {
            c = t->child[i];
            t->child[i] = t->child[t->nchild - 1];
            t->child_idx[i] = t->child_idx[t->nchild - 1];
            t->nchild--;
            break;
        }
    }
    if (!c) { fprintf(stderr, "oracle: traverse to non-existent child\n"); abort(); }
    mct_free(t);
    for (int i = 0; i < c->nchild; i++) mct_free(c->child[i]);   /* drop grandchildren */
    c->nchild = 0;
    if (noise) apply_dirichlet_noise(cfg, c->policy, c->moves, c->nmoves, key);
    memset(c->visits, 0, sizeof(float) * REF_ACTION_SPACE);
    memset(c->scores, 0, sizeof(float) * REF_ACTION_SPACE);
    return c;
}

/* ---------------- single search (for parity tests) ---------------- */

int ref_search_game(const ref_search_cfg* cfg, const ref_replay* rep, const int32_t* history, int nhist,
                    int noise, uint64_t noise_key, ref_search_out* out) {
    return ref_search_from(cfg, rep, NULL, history, nhist, noise, noise_key, out);
}

int ref_search_from(const ref_search_cfg* cfg, const ref_replay* rep, const ref_pos* start, const int32_t* history,
                    int nhist, int noise, uint64_t noise_key, ref_search_out* out) {
    ref_game g;
    if (start) ref_game_from(&g, start);
    else ref_game_new(&g);
    for (int i = 0; i < nhist; i++) {
        ref_move m;
        if (!ref_index_to_move(history[i], &g.position, &m)) { ref_game_free(&g); return -1; }
        if (ref_play_move(&g, m) != REF_ONGOING) { ref_game_free(&g); return -2; }
    }
    eval_ctx ctx = {cfg, rep, 0, 0};
    float* policy = (float*)malloc(sizeof(float) * REF_ACTION_SPACE);
    float v;
    evaluate(&ctx, &g.position, policy, &v);
    mct* t = mct_new(cfg, policy, &g, noise, noise_key);
    free(policy);
    mct_search(t, &ctx, out);
    out->evals = ctx.evals;
    mct_free(t);
    ref_game_free(&g);
    return ctx.failed ? -3 : 0;
}

/* ---------------- self-play (training.rs:294-378) ---------------- */

static int argmax_last(const float* v) {       /* Iterator::max_by: last of equal maxima */
    int best = 0;
    for (int i = 1; i < REF_ACTION_SPACE; i++) if (!(v[i] < v[best])) best = i;
    return best;
}

/* rand 0.8.5 WeightedIndex: cumulative f32 sums, first cumulative weight > x */
static int weighted_index(const float* w, float u) {
    float total = w[0];
    float cw[REF_ACTION_SPACE];
    for (int i = 1; i < REF_ACTION_SPACE; i++) { cw[i - 1] = total; total += w[i]; }
    float x = u * total;
    if (!(x < total)) x = nextafterf(total, 0.0f);
    int lo = 0, hi = REF_ACTION_SPACE - 1;                         /* partition_point(cw <= x) */
    while (lo < hi) { int mid = (lo + hi) / 2; if (cw[mid] <= x) lo = mid + 1; else hi = mid; }
    return lo;
}

typedef struct {
    int32_t ply, action, depth, result;
    float turn;
    uint64_t key;
    int32_t nvis;
    int32_t vis_idx[256];
    float vis_n[256];
} step_tmp;

static int run_episode(const ref_search_cfg* cfg, const ref_replay* rep, int game_id, int max_plies,
                       const float* start_policy, step_tmp* hist, int* nhist, float* final_scale,
                       int64_t* sims, int64_t* evals, int* failed) {
    eval_ctx ctx = {cfg, rep, 0, 0};
    ref_game state;
    ref_game_new(&state);
    mct* tree = mct_new(cfg, start_policy, &state, cfg->noise, ref_stream_key(cfg->seed, (uint64_t)game_id, 0, 0));
    ref_search_out* so = (ref_search_out*)malloc(sizeof(ref_search_out));
    int ply = 0, result_code = REF_ONGOING;
    float result = 0.0f;
    *nhist = 0;
    for (;;) {
        mct_search(tree, &ctx, so);
        *sims += cfg->sims;
        float turn = state.position.turn == 0 ? 1.0f : -1.0f;
        step_tmp* st = &hist[(*nhist)++];
        st->ply = ply; st->depth = so->depth; st->turn = turn; st->key = ref_fen_key(&state.position);
        st->nvis = 0;
        for (int i = 0; i < REF_ACTION_SPACE; i++)
            if (so->visits[i] != 0.0f && st->nvis < 256) { st->vis_idx[st->nvis] = i; st->vis_n[st->nvis] = so->visits[i]; st->nvis++; }
        int action;
        if ((uint32_t)state.position.fullmoves >= (uint32_t)cfg->temp_moves) {
            action = argmax_last(so->improved);                    /* training.rs:310-317 */
        } else {
            uint64_t ctr = 0;
            float u = ref_uniform01(ref_stream_key(cfg->seed, (uint64_t)game_id, (uint64_t)ply, 1), &ctr);
            action = weighted_index(so->improved, u);              /* training.rs:318-321 */
        }
        st->action = action;
        ref_move m;
        if (!ref_index_to_move(action, &state.position, &m)) { fprintf(stderr, "oracle: model played illegal move\n"); abort(); }
        int r = ref_play_move(&state, m);
        ply++;
        if (r == REF_ONGOING) {
            if (max_plies > 0 && ply >= max_plies) { result_code = -2; break; }
            tree = mct_traverse_new(tree, action, cfg, cfg->noise,
                                    ref_stream_key(cfg->seed, (uint64_t)game_id, (uint64_t)ply, 0));
            continue;
        }
        if (r == REF_DRAW) { result = 0.0f; result_code = REF_DRAW; }
        else { result = turn; result_code = r; }
        break;
    }
    float decay = 1.0f - ((float)state.position.fullmoves / (2.0f * (float)REF_NUM_FULLMOVES));
    *final_scale = result * decay;
    for (int i = 0; i < *nhist; i++) hist[i].result = result_code;
    if (result_code == -2) *final_scale = 0.0f;
    mct_free(tree);
    ref_game_free(&state);
    free(so);
    *evals += ctx.evals;
    if (ctx.failed) *failed = 1;
    return result_code;
}

int64_t ref_selfplay(const ref_search_cfg* cfg, const ref_replay* rep, int ngames, int max_plies,
                     ref_step* steps, int64_t cap, int64_t* sims_done, int64_t* evals_done) {
    /* shared root evaluation of the start position (training.rs:344-350) */
    eval_ctx ctx0 = {cfg, rep, 0, 0};
    ref_game g0;
    ref_game_new(&g0);
    float* start_policy = (float*)malloc(sizeof(float) * REF_ACTION_SPACE);
    float v0;
    evaluate(&ctx0, &g0.position, start_policy, &v0);
    ref_game_free(&g0);
    int64_t total_sims = 0, total_evals = ctx0.evals;
    int any_failed = ctx0.failed;
    int maxp = max_plies > 0 ? max_plies : 512;
    step_tmp** hists = (step_tmp**)calloc((size_t)ngames, sizeof(step_tmp*));
    int* nh = (int*)calloc((size_t)ngames, sizeof(int));
    float* scale = (float*)calloc((size_t)ngames, sizeof(float));
#pragma omp parallel for schedule(dynamic, 1) num_threads(cfg->threads > 0 ? cfg->threads : 1) reduction(+:total_sims, total_evals)
    for (int g = 0; g < ngames; g++) {
        int64_t s = 0, e = 0;
        int failed = 0;
        hists[g] = (step_tmp*)malloc(sizeof(step_tmp) * (size_t)maxp);
        run_episode(cfg, rep, g, max_plies, start_policy, hists[g], &nh[g], &scale[g], &s, &e, &failed);
        total_sims += s; total_evals += e;
        if (failed) any_failed = 1;
    }
    int64_t n = 0;
    for (int g = 0; g < ngames; g++) {
        for (int i = 0; i < nh[g]; i++) {
            if (n < cap && steps) {
                step_tmp* st = &hists[g][i];
                ref_step* o = &steps[n];
                o->game = g; o->ply = st->ply; o->action = st->action; o->depth = st->depth;
                o->final_value = st->turn * scale[g];               /* training.rs:332-335 */
                o->result = st->result; o->fen_key = st->key; o->nvis = st->nvis;
                memcpy(o->vis_idx, st->vis_idx, sizeof(o->vis_idx));
                memcpy(o->vis_n, st->vis_n, sizeof(o->vis_n));
            }
            n++;
        }
        free(hists[g]);
    }
    free(hists); free(nh); free(scale); free(start_policy);
    if (sims_done) *sims_done = total_sims;
    if (evals_done) *evals_done = total_evals;
    return any_failed ? -1 : n;
}

/* ---------------- arena and Elo (validation.rs, ratings.rs) ---------------- */

/* validation.rs:297-308 / 336-346: fullmoves > num_stochastic_moves (strict) -> the last maximal
 * index (Iterator::max_by over partial_cmp), else WeightedIndex::new(policy).sample() with the
 * uniform draw u standing in for thread_rng */
int ref_arena_choose(const float* policy, int fullmoves, int num_stochastic_moves, float u) {
    if (fullmoves > num_stochastic_moves) return argmax_last(policy);
    return weighted_index(policy, u);
}

/* validation.rs:325-335: the base-model player zeroes every index not produced by a legal move */
void ref_mask_to_legal(const ref_pos* p, float* policy) {
    ref_move mv[REF_MAX_MOVES];
    const int n = ref_legal_moves(p, mv);
    unsigned char legal[REF_ACTION_SPACE];
    memset(legal, 0, sizeof(legal));
    for (int i = 0; i < n; i++) legal[ref_move_to_index(mv[i], p->turn)] = 1;
    for (int i = 0; i < REF_ACTION_SPACE; i++) if (!legal[i]) policy[i] = 0.0f;
}

/* ratings.rs:113-144: fixed-point Elo fit, f32, LEARNING_RATE 8, 1000 iterations, player 0
 * pinned at base_elo; expected score 1 / (1 + 10^((prev[j] - prev[i]) / 400)) */
void ref_compute_elos(const float* wm, int n, float base_elo, float* elos) {
    float prev[64];
    for (int i = 0; i < n; i++) elos[i] = base_elo;
    for (int it = 0; it < 1000; it++) {
        for (int i = 0; i < n; i++) prev[i] = elos[i];
        for (int i = 1; i < n; i++) {
            float actual = 0.0f, expected = 0.0f;
            for (int j = 0; j < n; j++) {
                if (i == j) continue;
                actual += wm[i * n + j];
                const float diff = prev[j] - prev[i];
                expected += 1.0f / (1.0f + powf(10.0f, diff / 400.0f));
            }
            elos[i] += 8.0f * (actual - expected);
        }
    }
}

/* ---------------- batched lockstep self-play (CPU baseline) ----------------
 * The reference's self-play structure on the host -- one task per game, each with ONE outstanding
 * leaf, a batcher running one forward over every pending request (training.rs:340-422) -- in
 * lockstep: per simulation step every game selects its leaf (tree.rs:117-132, same dense-4096
 * trees as above, OpenMP over games), the leaves that need the network go through ONE batched
 * evaluation (to_tensor planes in, softmax rows + values out: process_batch), then every game
 * inserts its child and backs up (tree.rs:134-143).  A game's simulations stay sequential, so
 * its results equal run_episode's bit for bit given the same evaluations (tests/
 * test_oracle_rules_data.py).  fn == NULL evaluates through cfg->eval_kind instead. */
typedef struct {
    mct** node;
    int32_t* idx;
    int len;
    ref_game leaf;
    int kind;              /* 0 needs the network, 1 draw, 2 the mover won */
    int row;
} pend_leaf;

static void batched_select(mct* t, const ref_search_cfg* cfg, pend_leaf* p) {
    p->len = 0;
    for (;;) {
        float max_value = -INFINITY, total_visits = 0.0f;
        int max_index = 0;
        for (int i = 0; i < REF_ACTION_SPACE; i++) total_visits += t->visits[i];
        total_visits = total_visits + 1.0f;                            /* tree.rs:121 */
        for (int k = 0; k < t->nmoves; k++) {                          /* tree.rs:123-132 */
            int i = t->moves[k];
            float u_value = cfg->c_puct * t->policy[i] * sqrtf(total_visits) / (1.0f + t->visits[i]);
            float q_value = t->visits[i] > 0.0f ? t->scores[i] / t->visits[i] : 0.0f;
            float value = q_value + u_value;
            if (value > max_value) { max_value = value; max_index = i; }
        }
        p->node[p->len] = t;
        p->idx[p->len] = max_index;
        p->len++;
        mct* c = mct_find(t, max_index);
        if (c) { t = c; continue; }
        ref_game_clone(&p->leaf, &t->state);                           /* tree.rs:210-212 */
        ref_move m;
        if (!ref_index_to_move(max_index, &p->leaf.position, &m)) { fprintf(stderr, "oracle: Illegal move!\n"); abort(); }
        int r = ref_play_move(&p->leaf, m);
        p->kind = r == REF_ONGOING ? 0 : (r == REF_DRAW ? 1 : 2);
        return;
    }
}

static void batched_finish(pend_leaf* p, const ref_search_cfg* cfg, const float* policy, float nn_value) {
    float v;                                                           /* the leaf's value, its mover's view */
    mct* last = p->node[p->len - 1];
    if (p->kind == 0) {
        mct_insert(last, p->idx[p->len - 1], mct_new(cfg, policy, &p->leaf, 0, 0));
        v = nn_value;
    } else {
        v = p->kind == 1 ? 0.0f : -1.0f;                               /* tree.rs:233-234 */
    }
    ref_game_free(&p->leaf);
    float value = -v;                                                  /* value = -child value per level */
    for (int l = p->len - 1; l >= 0; l--) {
        p->node[l]->scores[p->idx[l]] += value;
        p->node[l]->visits[p->idx[l]] += 1.0f;
        value = -value;
    }
}

typedef struct {
    ref_game state;
    mct* tree;
    int ply, active, nh, result_code;
    float scale;
    step_tmp* hist;
} batched_game;

int64_t ref_selfplay_batched(const ref_search_cfg* cfg, int ngames, int max_plies, ref_eval_batch_fn fn, void* ctx,
                             ref_step* steps, int64_t cap, int64_t* sims_done, int64_t* evals_done) {
    const int S = cfg->sims, threads = cfg->threads > 0 ? cfg->threads : 1;
    const int maxp = max_plies > 0 ? max_plies : 512;
    eval_ctx ectx = {cfg, NULL, 0, 0};
    float* pol = (float*)malloc(sizeof(float) * REF_ACTION_SPACE * (size_t)(ngames > 0 ? ngames : 1));
    float* val = (float*)malloc(sizeof(float) * (size_t)(ngames > 0 ? ngames : 1));
    float* planes = (float*)malloc(sizeof(float) * 19 * 64 * (size_t)(ngames > 0 ? ngames : 1));
    int* rows = (int*)malloc(sizeof(int) * (size_t)(ngames > 0 ? ngames : 1));
    int64_t total_sims = 0, total_evals = 0;
    int failed = 0;
    /* shared root evaluation of the start position (training.rs:344-350) */
    batched_game* gm = (batched_game*)calloc((size_t)ngames, sizeof(batched_game));
    ref_game g0;
    ref_game_new(&g0);
    if (fn) {
        ref_to_tensor(&g0.position, planes);
        failed |= fn(ctx, planes, 1, pol, val) != 0;
    } else {
        evaluate(&ectx, &g0.position, pol, val);
    }
    total_evals++;
    ref_game_free(&g0);
    for (int g = 0; g < ngames; g++) {
        ref_game_new(&gm[g].state);
        gm[g].tree = mct_new(cfg, pol, &gm[g].state, cfg->noise, ref_stream_key(cfg->seed, (uint64_t)g, 0, 0));
        gm[g].active = 1;
        gm[g].hist = (step_tmp*)malloc(sizeof(step_tmp) * (size_t)maxp);
    }
    pend_leaf* pl = (pend_leaf*)calloc((size_t)ngames, sizeof(pend_leaf));
    for (int g = 0; g < ngames; g++) {
        pl[g].node = (mct**)malloc(sizeof(mct*) * (size_t)(S + 2));
        pl[g].idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)(S + 2));
    }
    ref_search_out* so = (ref_search_out*)malloc(sizeof(ref_search_out) * (size_t)(ngames > 0 ? ngames : 1));
    for (;;) {
        int live = 0;
        for (int g = 0; g < ngames; g++) live += gm[g].active;
        if (!live) break;
        for (int s = 0; s < S && !failed; s++) {
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads)
            for (int g = 0; g < ngames; g++)
                if (gm[g].active) batched_select(gm[g].tree, cfg, &pl[g]);
            int n = 0;                                                 /* the batcher's requests */
            for (int g = 0; g < ngames; g++)
                if (gm[g].active && pl[g].kind == 0) { pl[g].row = n; rows[n++] = g; }
            if (n) {
                if (fn) {
#pragma omp parallel for num_threads(threads)
                    for (int r = 0; r < n; r++) ref_to_tensor(&pl[rows[r]].leaf.position, planes + (size_t)r * 19 * 64);
                    failed |= fn(ctx, planes, n, pol, val) != 0;       /* process_batch: one forward */
                } else {
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
                    for (int r = 0; r < n; r++) {
                        eval_ctx c = {cfg, NULL, 0, 0};
                        evaluate(&c, &pl[rows[r]].leaf.position, pol + (size_t)r * REF_ACTION_SPACE, val + r);
                    }
                }
                total_evals += n;
            }
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads)
            for (int g = 0; g < ngames; g++) {
                if (!gm[g].active) continue;
                const int r = pl[g].kind == 0 ? pl[g].row : 0;
                batched_finish(&pl[g], cfg, pol + (size_t)r * REF_ACTION_SPACE, pl[g].kind == 0 ? val[r] : 0.0f);
            }
            total_sims += live;
        }
        if (failed) break;
        /* per move: improved policy, record, action choice, play, re-root (run_episode, training.rs:294-338) */
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
        for (int g = 0; g < ngames; g++) {
            batched_game* G = &gm[g];
            if (!G->active) continue;
            mct* t = G->tree;
            float sum = 0.0f;
            for (int i = 0; i < REF_ACTION_SPACE; i++) sum += t->visits[i];
            for (int i = 0; i < REF_ACTION_SPACE; i++) { so[g].visits[i] = t->visits[i]; so[g].improved[i] = t->visits[i] / sum; }
            so[g].depth = mct_depth(t);
            float turn = G->state.position.turn == 0 ? 1.0f : -1.0f;
            step_tmp* st = &G->hist[G->nh++];
            st->ply = G->ply; st->depth = so[g].depth; st->turn = turn; st->key = ref_fen_key(&G->state.position);
            st->nvis = 0;
            for (int i = 0; i < REF_ACTION_SPACE; i++)
                if (so[g].visits[i] != 0.0f && st->nvis < 256) { st->vis_idx[st->nvis] = i; st->vis_n[st->nvis] = so[g].visits[i]; st->nvis++; }
            int action;
            if ((uint32_t)G->state.position.fullmoves >= (uint32_t)cfg->temp_moves) {
                action = argmax_last(so[g].improved);
            } else {
                uint64_t c = 0;
                float u = ref_uniform01(ref_stream_key(cfg->seed, (uint64_t)g, (uint64_t)G->ply, 1), &c);
                action = weighted_index(so[g].improved, u);
            }
            st->action = action;
            ref_move m;
            if (!ref_index_to_move(action, &G->state.position, &m)) { fprintf(stderr, "oracle: model played illegal move\n"); abort(); }
            int r = ref_play_move(&G->state, m);
            G->ply++;
            if (r == REF_ONGOING && !(max_plies > 0 && G->ply >= max_plies)) {
                G->tree = mct_traverse_new(G->tree, action, cfg, cfg->noise,
                                           ref_stream_key(cfg->seed, (uint64_t)g, (uint64_t)G->ply, 0));
                continue;
            }
            float result = 0.0f;
            if (r == REF_ONGOING) G->result_code = -2;
            else if (r == REF_DRAW) G->result_code = REF_DRAW;
            else { result = turn; G->result_code = r; }
            float decay = 1.0f - ((float)G->state.position.fullmoves / (2.0f * (float)REF_NUM_FULLMOVES));
            G->scale = G->result_code == -2 ? 0.0f : result * decay;
            for (int i = 0; i < G->nh; i++) G->hist[i].result = G->result_code;
            mct_free(G->tree);
            G->tree = NULL;
            G->active = 0;
        }
    }
    int64_t n = 0;
    for (int g = 0; g < ngames; g++) {
        for (int i = 0; i < gm[g].nh; i++) {
            if (n < cap && steps) {
                step_tmp* st = &gm[g].hist[i];
                ref_step* o = &steps[n];
                o->game = g; o->ply = st->ply; o->action = st->action; o->depth = st->depth;
                o->final_value = st->turn * gm[g].scale;
                o->result = st->result; o->fen_key = st->key; o->nvis = st->nvis;
                memcpy(o->vis_idx, st->vis_idx, sizeof(o->vis_idx));
                memcpy(o->vis_n, st->vis_n, sizeof(o->vis_n));
            }
            n++;
        }
        if (gm[g].tree) mct_free(gm[g].tree);
        ref_game_free(&gm[g].state);
        free(gm[g].hist);
        free(pl[g].node); free(pl[g].idx);
    }
    free(gm); free(pl); free(so); free(pol); free(val); free(planes); free(rows);
    if (sims_done) *sims_done = total_sims;
    if (evals_done) *evals_done = total_evals;
    return failed ? -1 : n;
}

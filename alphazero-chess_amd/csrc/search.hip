// search.hip -- GPU-resident batched MCTS (tree.rs) and self-play driver (training.rs).
//
// All G games advance in lockstep: one simulation step = for every game
//   k_select  (1 wavefront / game): walk root -> leaf over the struct-of-arrays tree,
//             PUCT u = C*P*sqrt(Nt)/(1+N), q = N>0 ? W/N : 0 (tree.rs:117-132, same f32
//             operation order, -ffp-contract=off), wave-reduce argmax taking the FIRST
//             max in `moves` order (strict '>' in the reference);
//   k_expand  (1 wavefront / game): index_to_move + play_move (chess.rs:36-63): legal move
//             generation of the child (its edge list), outcome(), repetition count over
//             the tree path + game history, 50-move / 200-fullmove draws; non-terminal
//             leaves become a node and a network row (tree.rs:146-167, 209-237);
//   evaluation of all new rows in one batch (process_batch, training.rs:380-422):
//             encode -> conv tower -> fused heads writing legal priors into the edges;
//   k_backup  (1 wavefront / game, one lane per tree level): W += +-v, N += 1
//             (tree.rs:134-143, 197-206).
// Outside the timed (event-bracketed) steps the three tree kernels run as ONE launch,
// k_step: backup of step i-1, select and expand of step i, one wavefront per game (the
// expansion wave-parallel), so a simulation step is two launches: k_step and the tower.
// A move step (k_finish) computes the improved policy visits/sum (tree.rs:110-114),
// chooses the action (argmax with the LAST max at fullmoves >= 15, else WeightedIndex
// over f32 cumulative sums: training.rs:310-321), records the EpisodeStep, plays it and
// re-roots on the child keeping its priors/edges but resetting N/W and dropping every
// other node (traverse_new, tree.rs:239-256), then applies Dirichlet noise
// (tree.rs:272-289).  Nothing crosses PCIe inside a move.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <vector>

#include "az_internal.h"
#include "detmath.h"
#include "search_dev.h"

#pragma clang fp contract(off)

namespace azi {

__global__ void __launch_bounds__(256) k_select(Engine E) {
    const int g = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (g >= E.G || !E.active[g]) return;
    select_game(E, g, threadIdx.x & 63);
}

// insert every row just evaluated by the network (process_batch's cache.insert, training.rs:413)
__global__ void __launch_bounds__(64) k_cache_insert(Engine E, int step) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= load_fresh(step_rows(E, step))) return;
    const int g = E.row_game[row], node = E.row_node[row];
    const azc::Pos p = E.npos[(size_t)g * E.NMAX + node];
    const Node nd = E.nodes[(size_t)g * E.NMAX + node];
    const Edge* edges = E.edges + (size_t)g * E.EMAX + nd.edge_begin;
    const uint64_t key = azc::fen_key(p);
    int sl = -1;
    for (int i = 0; i < CACHE_PROBES && sl < 0; i++) {
        const int s = (int)((key + (uint64_t)i) & (uint64_t)E.cache_mask);
        const unsigned st = E.c_state[s];
        if (st == 2u && E.c_key[s] == key && same_fen(E.c_pos[s], p)) return;   // already cached
        if (st == 0u && atomicCAS(&E.c_state[s], 0u, 1u) == 0u) sl = s;
    }
    if (sl < 0) {                                            // all probes taken: replace the first
        const int s = (int)(key & (uint64_t)E.cache_mask);
        if (atomicCAS(&E.c_state[s], 2u, 1u) != 2u) return;  // another row is writing it: skip
        sl = s;
    }
    E.c_key[sl] = key;
    E.c_pos[sl] = p;
    E.c_value[sl] = E.value[row];
    E.c_n[sl] = nd.nedges;
    float* pri = E.c_pri + (size_t)sl * MAX_EDGES;
    for (int e = 0; e < nd.nedges; e++) pri[e] = edges[e].P;
    __threadfence();
    atomicExch(&E.c_state[sl], 2u);
}



// one wavefront per game (expand_leaf_wave); the row allocation on lane 0
__global__ void __launch_bounds__(64) k_expand(Engine E, int step) {
    const int lane = threadIdx.x;
    const int g = vgpr_index(blockIdx.x);
    int nid = -1;
    const int kind = expand_leaf_wave(E, g, lane, &nid);
    if (lane == 0) {
        if (kind == X_ROW) {
            const int row = atomicAdd(step_rows(E, step), 1);
            E.row_game[row] = g;
            E.row_node[row] = nid;
            E.leaf_row[g] = row;
        } else if (kind == X_TERMINAL) {
            atomicAdd(&E.ctr->terminal, 1ull);
        } else if (kind == X_CACHED) {
            atomicAdd(&E.ctr->cache_hits, 1ull);
        }
    }
}


__global__ void __launch_bounds__(256) k_backup(Engine E, int step) {
    const int g = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (g == 0 && lane == 0) backup_stats(E, step);
    if (g >= E.G || !E.active[g]) return;
    backup_game(E, g, lane);
}

// ------------------------------------------------------------------ fused step
// One launch per simulation step instead of three: backup of step `bstep` (the previous one,
// or none when < 0), then select and expand of step `step`, one wavefront per game (the
// expansion wave-parallel).  A game's backup, select and expand touch only that game's tree, so
// the wave needs no grid-wide order; the wave's own global stores (backup) are made visible
// to its later loads (select) by a workgroup-scope fence.  Rows are allocated with one atomic
// per workgroup (STEP_WPB games).  bstep's row counter is read and cleared by one thread;
// step's counter (the other parity) was cleared by the backup of step - 2.
#ifndef AZ_STEP_WPB
#define AZ_STEP_WPB 1      // C2 A/B (profiles/r02_ab_movegen_c2_*.log): 1 wave per workgroup +2.5 % over 4 (no barrier wait on the slowest game)
#endif
constexpr int STEP_WPB = AZ_STEP_WPB;   // games (waves) per k_step workgroup
static_assert(STEP_WPB <= GEN_WAVES, "gen_legal_wave stages moves in LDS for at most GEN_WAVES waves");
#ifdef AZ_STEP_TRACE   // experiment: per-wave phase stamps of step AZ_STEP_TRACE (tools/step_trace.py)
#define ST_STAMP(k) do { if (step == AZ_STEP_TRACE && lane == 0 && g < E.G) E.trace[(size_t)g * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define ST_STAMP(k) do { } while (0)
#endif
__global__ void __launch_bounds__(STEP_WPB * 64) k_step(Engine E, int step, int bstep) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = blockIdx.x * STEP_WPB + w;
    __shared__ int s_kind[STEP_WPB], s_nid[STEP_WPB], s_base;
    ST_STAMP(0);
    const bool live = g < E.G && E.active[g];
    if (bstep >= 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) backup_stats(E, bstep);
        if (live) backup_game(E, g, lane);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    ST_STAMP(1);
    int kind = X_NONE, nid = -1;
    if (live) {
        select_game(E, g, lane);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        ST_STAMP(2);
        kind = expand_leaf_wave(E, g, lane, &nid, step);
    }
    ST_STAMP(3);
    if (lane == 0) { s_kind[w] = kind; s_nid[w] = nid; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int nr = 0, nt = 0, nc = 0;
        for (int i = 0; i < STEP_WPB; i++) {
            nr += s_kind[i] == X_ROW;
            nt += s_kind[i] == X_TERMINAL;
            nc += s_kind[i] == X_CACHED;
        }
        s_base = nr ? atomicAdd(step_rows(E, step), nr) : 0;
        if (nt) atomicAdd(&E.ctr->terminal, (unsigned long long)nt);
        if (nc) atomicAdd(&E.ctr->cache_hits, (unsigned long long)nc);
    }
    __syncthreads();
    if (lane == 0 && kind == X_ROW) {
        int row = s_base;
        for (int i = 0; i < w; i++) row += s_kind[i] == X_ROW;
        E.row_game[row] = g;
        E.row_node[row] = nid;
        E.leaf_row[g] = row;
    }
    ST_STAMP(4);
}

// ------------------------------------------------------------------ roots
// root node from hist[g][hist_len-1]; every game gets batch row g
__global__ void __launch_bounds__(64) k_root_setup(Engine E) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= E.G || !E.active[g]) return;
    Edge* edges = game_edges(E, g);
    const azc::Pos p = E.hist[(size_t)g * HMAX + E.hist_len[g] - 1];
    EdgeSink sink{edges, 0};
    bool chk, lep;
    const int n = azc::gen_legal(p, sink, &chk, &lep);
    Node nd;
    nd.edge_begin = 0; nd.nedges = (uint16_t)n; nd.depth = 0; nd.nsum = 0; nd.parent = -1;
    game_nodes(E, g)[0] = nd;
    game_npos(E, g)[0] = p;
    E.node_count[g] = 1;
    E.edge_count[g] = n;
    E.max_depth[g] = 0;
    const int row = atomicAdd(&E.ctr->batch_count[0], 1);   // cleared again after the root eval
    E.row_game[row] = g;
    E.row_node[row] = 0;
}

// Dirichlet noise on the root priors (tree.rs:272-289).  One 64-thread block per game.
__device__ void root_noise(const Engine& E, int g, int gid, int ply, float* gam, int* kpos, float* sh) {
    const int lane = threadIdx.x;
    Edge* edges = game_edges(E, g);
    const int n = game_nodes(E, g)[0].nedges;
    if (lane == 0) {
        int run = 0;
        for (int e = 0; e < n; e++) { kpos[e] = run; run += (edges[e].idx & azc::PROMO_FLAG) ? 4 : 1; }
        kpos[n] = run;
    }
    __syncthreads();
    const int ns = kpos[n];                 // len(moves) including under-promotion duplicates
    if (ns < 2) return;
    const uint64_t key = azc::stream_key(E.seed, (uint64_t)gid, (uint64_t)ply, 0);
    for (int k = lane; k < ns; k += 64) gam[k] = azc::gamma_sample(E.dir_alpha, azc::dirichlet_component_key(key, k));
    __syncthreads();
    if (lane == 0) {
        float sum = 0.0f;
        for (int k = 0; k < ns; k++) sum = sum + gam[k];
        sh[0] = 1.0f / sum;
    }
    __syncthreads();
    const float inv = sh[0];
    const float keep = 1.0f - E.dir_eps;
    for (int e = lane; e < n; e += 64) {
        float P = edges[e].P * keep;
        const int dup = (edges[e].idx & azc::PROMO_FLAG) ? 4 : 1;
        for (int j = 0; j < dup; j++) P = P + E.dir_eps * (gam[kpos[e] + j] * inv);
        edges[e].P = P;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(64) k_root_noise(Engine E, int apply) {
    __shared__ float gam[AZ_MAX_MOVES];
    __shared__ int kpos[MAX_EDGES + 1];
    __shared__ float sh[2];
    const int g = vgpr_index(blockIdx.x);
    if (g >= E.G || !E.active[g] || !apply) return;
    root_noise(E, g, E.game_id[g], E.ply[g], gam, kpos, sh);
}

__global__ void k_save_start_template(Engine E) {   // game 0's un-noised startpos root
    const Edge* edges = game_edges(E, vgpr_index(0));
    const int n = game_nodes(E, vgpr_index(0))[0].nedges;
    for (int e = threadIdx.x; e < n; e += blockDim.x) E.start_edges[e] = edges[e];
    if (threadIdx.x == 0) *E.start_n = n;
}

// ------------------------------------------------------------------ move step
// mode 0: self-play (choose, record, restart); mode 1: advance with given actions.
__global__ void __launch_bounds__(64) k_finish(Engine E, int mode, const int* actions, int* results, int apply_noise) {
    __shared__ uint16_t s_idx[MAX_EDGES];
    __shared__ uint16_t s_n[MAX_EDGES];
    __shared__ float s_P[MAX_EDGES];
    __shared__ float gam[AZ_MAX_MOVES];
    __shared__ int kpos[MAX_EDGES + 1];
    __shared__ float sh[2];
    __shared__ int si[4];
    const int g = vgpr_index(blockIdx.x), lane = threadIdx.x;
    if (g >= E.G || !E.active[g]) return;
    Node* nodes = game_nodes(E, g);
    Edge* edges = game_edges(E, g);
    azc::Pos* npos = game_npos(E, g);
    azc::Pos* hist = E.hist + (size_t)g * HMAX;
    const int hl = E.hist_len[g];
    const azc::Pos root = hist[hl - 1];
    const int n = nodes[0].nedges;
    const int gid = E.game_id[g], ply = E.ply[g];
    int action = -1;
    if (mode == 0) {
        // improved policy = visits / sum(visits) (T = 1, tree.rs:110-114)
        int tot = 0;
        for (int e = lane; e < n; e += 64) tot += edges[e].N;
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (root.fullmoves >= E.temp_moves) {                 // training.rs:310-317, LAST max
            int bn = -1, bi = -1;
            for (int e = lane; e < n; e += 64) {
                const int nn = edges[e].N, ii = edges[e].idx & azc::IDX_MASK;
                if (nn > bn || (nn == bn && ii > bi)) { bn = nn; bi = ii; }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const int on = __shfl_xor(bn, o, 64), oi = __shfl_xor(bi, o, 64);
                if (on > bn || (on == bn && oi > bi)) { bn = on; bi = oi; }
            }
            action = bi;
        } else {                                               // training.rs:318-321
            for (int e = lane; e < n; e += 64) {
                const int ii = edges[e].idx & azc::IDX_MASK;
                int r = 0;
                for (int f = 0; f < n; f++) r += (edges[f].idx & azc::IDX_MASK) < ii;
                s_idx[r] = (uint16_t)ii;
                s_n[r] = edges[e].N;
            }
            __syncthreads();
            if (lane == 0) {
                const float totf = (float)tot;
                float total = 0.0f;
                for (int r = 0; r < n; r++) if (s_n[r]) total = total + (float)s_n[r] / totf;
                uint64_t ctr = 0;
                const float u = azc::uniform01(azc::stream_key(E.seed, (uint64_t)gid, (uint64_t)ply, 1), ctr);
                float x = u * total;
                if (!(x < total)) x = nextafterf(total, 0.0f);
                float cw = 0.0f;
                int a = -1, last = -1;
                for (int r = 0; r < n; r++) {
                    if (!s_n[r]) continue;
                    last = s_idx[r];
                    cw = cw + (float)s_n[r] / totf;
                    if (cw > x) { a = s_idx[r]; break; }
                }
                si[0] = a >= 0 ? a : last;
            }
            __syncthreads();
            action = si[0];
        }
        // EpisodeStep record (training.rs:303-308)
        if (lane == 0) si[1] = atomicAdd(&E.ctr->rec_count, 1);
        __syncthreads();
        const int rid = si[1];
        if (rid < E.rec_cap) {
            StepRec* R = E.recs + rid;
            for (int e = lane; e < n; e += 64) {
                R->vis_idx[e] = edges[e].idx & azc::IDX_MASK;
                R->vis_n[e] = edges[e].N;
            }
            if (lane == 0) {
                R->game_id = gid; R->ply = (int16_t)ply; R->action = (int16_t)action;
                R->depth = (int16_t)E.max_depth[g]; R->nvis = (int16_t)n; R->kind = 0; R->result = -1;
                R->end_fullmoves = 0; R->pos = root;
                atomicAdd(&E.ctr->moves, 1ull);
                atomicAdd(&E.ctr->depth_sum, (unsigned long long)E.max_depth[g]);
            }
        }
    } else {
        action = actions[g];
    }
    // locate the action's edge and play it (training.rs:323-329)
    if (lane == 0) si[2] = -1;
    __syncthreads();
    for (int e = lane; e < n; e += 64)
        if ((edges[e].idx & azc::IDX_MASK) == action) si[2] = e;
    __syncthreads();
    const int ea = si[2];
    const int child = ea >= 0 ? edges[ea].child : CHILD_NONE;
    if (child >= 0) {
        const azc::Pos cp = npos[child];
        const Node cn = nodes[child];
        for (int e = lane; e < cn.nedges; e += 64) {
            s_idx[e] = edges[cn.edge_begin + e].idx;
            s_P[e] = edges[cn.edge_begin + e].P;
        }
        __syncthreads();
        for (int e = lane; e < cn.nedges; e += 64) {
            Edge ne;
            ne.P = s_P[e]; ne.W = 0.0f; ne.N = 0; ne.idx = s_idx[e]; ne.child = CHILD_NONE;
            edges[e] = ne;
        }
        if (lane == 0) {
            Node r;
            r.edge_begin = 0; r.nedges = cn.nedges; r.depth = 0; r.nsum = 0; r.parent = -1;
            nodes[0] = r;
            npos[0] = cp;
            if (hl < HMAX) { hist[hl] = cp; E.hist_len[g] = hl + 1; }
            E.ply[g] = ply + 1;
            E.node_count[g] = 1;
            E.edge_count[g] = cn.nedges;
            E.max_depth[g] = 0;
            if (results) results[g] = azc::ONGOING;
        }
        __syncthreads();
        if (apply_noise) root_noise(E, g, gid, ply + 1, gam, kpos, sh);
        return;
    }
    // terminal move (or an action that was never expanded)
    int res;
    if (child == CHILD_DRAW) res = azc::DRAW;
    else if (child == CHILD_WIN) res = root.turn == 0 ? azc::WHITE_WINS : azc::BLACK_WINS;
    else res = azc::ILLEGAL;
    if (mode == 1) {
        if (lane == 0) { results[g] = res; E.active[g] = 0; }
        return;
    }
    if (lane == 0) {
        const int rid = atomicAdd(&E.ctr->rec_count, 1);
        if (rid < E.rec_cap) {
            StepRec* R = E.recs + rid;
            R->game_id = gid; R->ply = (int16_t)(ply + 1); R->action = (int16_t)action; R->depth = 0;
            R->nvis = 0; R->kind = 1; R->result = (int16_t)res;
            R->end_fullmoves = (int16_t)(ea >= 0 ? azc::play_index(root, action).fullmoves : root.fullmoves);
        }
        atomicAdd(&E.ctr->games_finished, 1ull);
    }
    if (!E.continuous) {
        if (lane == 0) E.active[g] = 0;
        return;
    }
    // new game in this slot from startpos (training.rs:353-358)
    if (lane == 0) si[3] = atomicAdd(&E.ctr->next_game_id, 1);
    __syncthreads();
    const int ngid = si[3];
    const int sn = load_fresh(E.start_n);
    for (int e = lane; e < sn; e += 64) edges[e] = E.start_edges[e];
    if (lane == 0) {
        const azc::Pos sp = azc::startpos();
        Node r;
        r.edge_begin = 0; r.nedges = (uint16_t)sn; r.depth = 0; r.nsum = 0; r.parent = -1;
        nodes[0] = r;
        npos[0] = sp;
        hist[0] = sp;
        E.hist_len[g] = 1;
        E.game_id[g] = ngid;
        E.ply[g] = 0;
        E.node_count[g] = 1;
        E.edge_count[g] = sn;
        E.max_depth[g] = 0;
    }
    __syncthreads();
    if (E.noise) root_noise(E, g, ngid, 0, gam, kpos, sh);
}

// ------------------------------------------------------------------ caller-owned evaluator
// AZ_EVAL_CALLBACK (the reference's InferenceRequest / process_batch, training.rs:28-31, 380-422):
// the rows' leaf positions go to the host in batch-row order, the caller's policy rows come back
// and are read at each new node's legal move indices (MCTree::new, tree.rs:84-104).
__global__ void __launch_bounds__(64) k_gather_rows(Engine E, const int* __restrict__ count_ptr, azc::Pos* out) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= load_fresh(count_ptr)) return;
    out[row] = E.npos[(size_t)E.row_game[row] * E.NMAX + E.row_node[row]];
}

__global__ void __launch_bounds__(64) k_apply_rows(const int* __restrict__ count_ptr, SearchOut so,
                                                   const float* __restrict__ policy, const float* __restrict__ value) {
    const int row = vgpr_index(blockIdx.x), lane = threadIdx.x;
    if (row >= load_fresh(count_ptr)) return;
    const int game = so.row_game[row], node = so.row_node[row];
    const Node nd = so.nodes[(size_t)game * so.NMAX + node];
    Edge* e = so.edges + (size_t)game * so.EMAX + nd.edge_begin;
    const float* pr = policy + (size_t)row * AZ_ACTION_SPACE;
    __shared__ int slot[2];
    if (lane == 0) {
        slot[0] = -1;
        if (so.log_cap > 0) {
            const int r = atomicAdd(&so.ctr->log_count, 1);
            const int po = atomicAdd(&so.ctr->log_prior_count, (int)nd.nedges);
            slot[0] = (r < so.log_cap && po + nd.nedges <= so.log_prior_cap) ? r : -1;
            slot[1] = po;
        }
    }
    __syncthreads();
    for (int i = lane; i < nd.nedges; i += 64) {
        const int idx = e[i].idx & azc::IDX_MASK;
        const float P = pr[idx];
        e[i].P = P;
        if (slot[0] >= 0) { so.log_idx[slot[1] + i] = idx; so.log_prior[slot[1] + i] = P; }
    }
    if (lane == 0) {
        so.value[row] = value[row];
        if (slot[0] >= 0) {
            so.log_key[slot[0]] = azc::fen_key(so.npos[(size_t)game * so.NMAX + node]);
            so.log_value[slot[0]] = value[row];
            so.log_off[slot[0]] = slot[1];
            so.log_n[slot[0]] = nd.nedges;
        }
    }
}

// visits / improved policy / depth readout (dense 4096 per game)
__global__ void k_readout(Engine E, float* improved, uint32_t* visits, int* depth) {
    const int g = vgpr_index(blockIdx.x);
    if (g >= E.G) return;
    const Node r = game_nodes(E, g)[0];
    const Edge* edges = game_edges(E, g);
    __shared__ int tot;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    int t = 0;
    for (int e = threadIdx.x; e < r.nedges; e += blockDim.x) t += edges[e].N;
    atomicAdd(&tot, t);
    for (int i = threadIdx.x; i < AZ_ACTION_SPACE; i += blockDim.x) {
        if (improved) improved[(size_t)g * AZ_ACTION_SPACE + i] = 0.0f;
        if (visits) visits[(size_t)g * AZ_ACTION_SPACE + i] = 0u;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < r.nedges; e += blockDim.x) {
        const int i = edges[e].idx & azc::IDX_MASK;
        if (improved) improved[(size_t)g * AZ_ACTION_SPACE + i] = (float)edges[e].N / (float)tot;
        if (visits) visits[(size_t)g * AZ_ACTION_SPACE + i] = edges[e].N;
    }
    if (threadIdx.x == 0 && depth) depth[g] = E.max_depth[g];
}

}  // namespace azi

// ====================================================================== host engine
#ifndef AZ_FUSED_STEPS
#define AZ_FUSED_STEPS 1
#endif
using namespace azi;

struct az_search {
    az_search_cfg cfg{};
    int device = 0;
    hipStream_t st = nullptr;
    az_net* net = nullptr;
    Engine E{};
    SearchOut so{};
    void* planes = nullptr; void* x = nullptr; void* h = nullptr;
    std::vector<void*> allocs;
    std::map<int, std::vector<StepRec>> pending;
    std::vector<az_episode_step> finished;
    size_t finished_read = 0;
    bool roots_fresh = false;        // trees sized for exactly S sims per root
    int sim_cursor = 0;              // simulation steps of the current self-play move already run
    // timing
    bool timing = false;
    bool fused_steps = AZ_FUSED_STEPS != 0;   // k_step (backup + select + expand in one launch); env AZ_FUSED_STEPS=0: separate kernels
    int persist = -1;                // k_sims32w (a game's whole simulation loop in one workgroup): -1 auto
                                     // (f32 Winograd or bf16 64-filter net, FEN cache off, G <= CUs), 0 off, 1 on; env AZ_PERSIST
    int cus = 256;                   // compute units of the device
    std::vector<hipEvent_t> ev;      // 7 per sim step
    az_timing acc{};
    // AZ_EVAL_CALLBACK: the caller's evaluator and its staging buffers (pinned host, device)
    az_eval_fn eval_fn = nullptr;
    void* eval_ctx = nullptr;
    azc::Pos* h_pos = nullptr; float* h_pol = nullptr; float* h_val = nullptr;
    azc::Pos* d_pos = nullptr; float* d_pol = nullptr; float* d_val = nullptr;
};

namespace {

template <typename T> int dalloc(az_search* s, T** p, size_t count) {
    void* q = nullptr;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    if (hipMalloc(&q, bytes) != hipSuccess) return fail("hipMalloc failed (" + std::to_string(bytes) + " B)");
    if (hipMemset(q, 0, bytes) != hipSuccess) return fail("hipMemset failed");
    s->allocs.push_back(q);
    *p = (T*)q;
    return 0;
}

constexpr int EV_PER_STEP = 9;
constexpr int TIMING_EVERY = 32;  // sampled simulation steps in timing mode (az_timing)

// sum of a per-game device counter (infrequent readouts; the stream is synchronised by the caller)
unsigned long long sum_games(az_search* s, const unsigned long long* d) {
    std::vector<unsigned long long> h(s->E.G);
    if (hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    unsigned long long t = 0;
    for (unsigned long long v : h) t += v;
    return t;
}

// AZ_EVAL_CALLBACK: the rows counted at *cnt (device) through the caller's evaluator -- one
// host round trip per simulation step, like the reference's batcher (training.rs:369-373)
int eval_callback(az_search* s, const int* cnt) {
    Engine& E = s->E;
    if (!s->eval_fn) return fail("AZ_EVAL_CALLBACK: no evaluator installed (az_search_set_evaluator)");
    int n = 0;
    AZ_HIP(hipMemcpyAsync(&n, cnt, 4, hipMemcpyDeviceToHost, s->st));
    AZ_HIP(hipStreamSynchronize(s->st));
    if (n < 0 || n > E.G) return fail("AZ_EVAL_CALLBACK: bad row count");
    if (n == 0) return 0;
    k_gather_rows<<<(n + 63) / 64, 64, 0, s->st>>>(E, cnt, s->d_pos);
    AZ_HIP(hipGetLastError());
    AZ_HIP(hipMemcpyAsync(s->h_pos, s->d_pos, (size_t)n * sizeof(azc::Pos), hipMemcpyDeviceToHost, s->st));
    AZ_HIP(hipStreamSynchronize(s->st));
    const int rc = s->eval_fn(s->eval_ctx, reinterpret_cast<const az_pos*>(s->h_pos), n, s->h_pol, s->h_val);
    if (rc != 0) return fail("AZ_EVAL_CALLBACK: the evaluator returned " + std::to_string(rc));
    AZ_HIP(hipMemcpyAsync(s->d_pol, s->h_pol, (size_t)n * AZ_ACTION_SPACE * 4, hipMemcpyHostToDevice, s->st));
    AZ_HIP(hipMemcpyAsync(s->d_val, s->h_val, (size_t)n * 4, hipMemcpyHostToDevice, s->st));
    k_apply_rows<<<n, 64, 0, s->st>>>(cnt, s->so, s->d_pol, s->d_val);
    AZ_HIP(hipGetLastError());
    return 0;
}

// network evaluation of step `step`'s rows (+ FEN cache insert); events 3, 7, 8, 4 when timed
int eval_step(az_search* s, int step, hipEvent_t* ev) {
    Engine& E = s->E;
    hipStream_t st = s->st;
    const int G = E.G;
    const int* cnt = &E.ctr->batch_count[step & 1];
    int rc = 0;
    if (s->cfg.evaluator == AZ_EVAL_NET) {
        NetDev* n = s->net->dev;
        const bool fused = n->fused && tower_supported(n);
        // the fused tower encodes its rows itself (planes = nullptr): no encode launch
        if (!fused) rc = net_encode_rows(n, E.npos, E.NMAX, E.row_game, E.row_node, cnt, G, s->planes, st);
        if (rc) return rc;
        if (ev) (void)hipEventRecord(ev[3], st);
        if (fused) {
            // one launch: to_tensor + 41 convs + heads, activations resident in LDS
            if (ev) (void)hipEventRecord(ev[7], st);
            rc = tower_forward(n, nullptr, cnt, G, nullptr, nullptr, &s->so, st);
            if (rc) return rc;
            if (ev) { (void)hipEventRecord(ev[8], st); (void)hipEventRecord(ev[4], st); }
        } else {
            rc = net_tower(n, s->planes, cnt, G, s->x, s->h, st, ev ? ev[7] : nullptr, ev ? ev[8] : nullptr);
            if (rc) return rc;
            if (ev) (void)hipEventRecord(ev[4], st);
            rc = net_heads_search(n, s->x, cnt, G, s->so, st);
            if (rc) return rc;
        }
    } else {
        if (ev) { (void)hipEventRecord(ev[3], st); (void)hipEventRecord(ev[7], st); (void)hipEventRecord(ev[8], st); }
        if (ev) (void)hipEventRecord(ev[4], st);
        rc = s->cfg.evaluator == AZ_EVAL_CALLBACK ? eval_callback(s, cnt) : synth_eval_rows(cnt, G, s->so, st);
        if (rc) return rc;
    }
    if (E.cache_mask >= 0) k_cache_insert<<<(G + 63) / 64, 64, 0, st>>>(E, step);
    return 0;
}

// one simulation step as separate kernels, bracketed by events when timed
int sim_step(az_search* s, int step, hipEvent_t* ev) {
    Engine& E = s->E;
    hipStream_t st = s->st;
    const int G = E.G;
    if (ev) (void)hipEventRecord(ev[0], st);
    k_select<<<(G * 64 + 255) / 256, 256, 0, st>>>(E);
    if (ev) (void)hipEventRecord(ev[1], st);
    k_expand<<<G, 64, 0, st>>>(E, step);
    if (ev) (void)hipEventRecord(ev[2], st);
    int rc = eval_step(s, step, ev);
    if (rc) return rc;
    if (ev) (void)hipEventRecord(ev[5], st);
    k_backup<<<(G * 64 + 255) / 256, 256, 0, st>>>(E, step);
    if (ev) (void)hipEventRecord(ev[6], st);
    return hipGetLastError() == hipSuccess ? 0 : fail("sim step launch failed");
}

// one simulation step through the fused kernel: backup of bstep (< 0: none), select + expand
// of step, then the evaluation; step's own backup is left to the next launch
int sim_step_fused(az_search* s, int step, int bstep) {
    Engine& E = s->E;
    k_step<<<(E.G + STEP_WPB - 1) / STEP_WPB, STEP_WPB * 64, 0, s->st>>>(E, step, bstep);
    int rc = eval_step(s, step, nullptr);
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : fail("sim step launch failed");
}

// evaluation of batch rows set up by k_root_setup (rows = games)
int eval_rows(az_search* s) {
    Engine& E = s->E;
    const int* cnt = &E.ctr->batch_count[0];
    if (s->cfg.evaluator == AZ_EVAL_NET) {
        NetDev* n = s->net->dev;
        if (n->fused && tower_supported(n)) return tower_forward(n, nullptr, cnt, E.G, nullptr, nullptr, &s->so, s->st);
        int rc = net_encode_rows(n, E.npos, E.NMAX, E.row_game, E.row_node, cnt, E.G, s->planes, s->st);
        if (!rc) rc = net_tower(n, s->planes, cnt, E.G, s->x, s->h, s->st, nullptr, nullptr);
        if (!rc) rc = net_heads_search(n, s->x, cnt, E.G, s->so, s->st);
        return rc;
    }
    if (s->cfg.evaluator == AZ_EVAL_CALLBACK) return eval_callback(s, cnt);
    return synth_eval_rows(cnt, E.G, s->so, s->st);
}

// k_sims32w for the untimed simulation steps: one workgroup per game, so only when the games fit
// the chip in one round (auto), never with the FEN cache (its inserts are a separate kernel)
bool use_persistent(const az_search* s) {
    if (s->persist == 0 || s->E.cache_mask >= 0 || s->cfg.evaluator != AZ_EVAL_NET) return false;
    const NetDev* n = s->net->dev;
    if (!n->fused || !sims_persistent_supported(n)) return false;
    return s->persist == 1 || s->E.G <= s->cus;
}

// simulation steps [i0, i1) of the current move (run_sims(s) = the whole move)
int run_sims(az_search* s, int i0 = 0, int i1 = -1) {
    const int S = s->E.S;
    if (i1 < 0) i1 = S;
    const bool tm = s->timing;
    if (tm && (int)s->ev.size() < EV_PER_STEP * S) {
        for (int i = (int)s->ev.size(); i < EV_PER_STEP * S; i++) {
            hipEvent_t e;
            AZ_HIP(hipEventCreate(&e));
            s->ev.push_back(e);
        }
    }
    // timing mode brackets every TIMING_EVERY-th simulation step with events (an event record
    // costs a few us of GPU time: on every step it was ~20 % of a 6x64 simulation step, on every
    // 8th still ~10 % of a bf16 one); those steps run as separate kernels, the others through the
    // fused step kernel
    int pending = -1;                  // step whose backup is still to launch
    const bool pers = use_persistent(s);
    for (int i = i0; i < i1; i++) {
        const bool timed = tm && i % TIMING_EVERY == 0;
        int rc;
        if (pers && !timed) {
            // the untimed steps up to the next timed one in one persistent launch (all backed up)
            int j = i + 1;
            while (j < i1 && !(tm && j % TIMING_EVERY == 0)) j++;
            if (pending >= 0) k_backup<<<(s->E.G * 64 + 255) / 256, 256, 0, s->st>>>(s->E, pending);
            pending = -1;
            rc = sims_persistent(s->net->dev, s->E, s->so, i, j, s->st);
            if (rc) return rc;
            i = j - 1;
            continue;
        }
        if (timed || !s->fused_steps) {
            if (pending >= 0) k_backup<<<(s->E.G * 64 + 255) / 256, 256, 0, s->st>>>(s->E, pending);
            pending = -1;
            rc = sim_step(s, i, timed ? &s->ev[EV_PER_STEP * i] : nullptr);
        } else {
            rc = sim_step_fused(s, i, pending);
            pending = i;
        }
        if (rc) return rc;
    }
    if (pending >= 0) k_backup<<<(s->E.G * 64 + 255) / 256, 256, 0, s->st>>>(s->E, pending);
    AZ_HIP(hipGetLastError());
#ifdef AZ_STEP_TRACE
    if (i0 <= AZ_STEP_TRACE && AZ_STEP_TRACE < i1) {
        std::vector<unsigned long long> h((size_t)s->E.G * 16);
        AZ_HIP(hipStreamSynchronize(s->st));
        AZ_HIP(hipMemcpy(h.data(), s->E.trace, h.size() * 8, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("AZ_STEP_TRACE_FILE") ? getenv("AZ_STEP_TRACE_FILE") : "step_trace.bin", "ab")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
#endif
    if (tm) {
        AZ_HIP(hipStreamSynchronize(s->st));
        std::vector<int> rows(S);
        AZ_HIP(hipMemcpy(rows.data(), s->E.batch_hist, S * 4, hipMemcpyDeviceToHost));
        const int first_timed = (i0 + TIMING_EVERY - 1) / TIMING_EVERY * TIMING_EVERY;
        const bool net = s->cfg.evaluator == AZ_EVAL_NET;
        const double F = net ? s->net->dev->filters : 0.0;
        const double per_row_conv = 2.0 * 64.0 * 9.0 * F * F;
        const double per_row_tower = net ? net_tower_flop_per_eval(s->net->dev->blocks, s->net->dev->filters) : 0.0;
        const bool fused = net && s->net->dev->fused && tower_supported(s->net->dev);
        for (int i = first_timed; i < i1; i += TIMING_EVERY) {
            hipEvent_t* e = &s->ev[EV_PER_STEP * i];
            float t[6], tc = 0.0f;
            for (int k = 0; k < 6; k++) (void)hipEventElapsedTime(&t[k], e[k], e[k + 1]);
            (void)hipEventElapsedTime(&tc, e[7], e[8]);
            az_timing& a = s->acc;
            a.select_ms += t[0]; a.select_launches++;
            a.expand_ms += t[1];
            a.encode_ms += t[2];
            a.tower_ms += t[3];
            a.heads_ms += t[4];
            a.backup_ms += t[5];
            a.sim_step_ms += t[0] + t[1] + t[2] + t[3] + t[4] + t[5];
            a.sim_steps++;
            a.rows += rows[i];
            if (net && rows[i] > 0 && s->net->dev->blocks > 0) {
                a.conv_ms += tc; a.conv_launches++;
                a.conv_flop += (fused ? per_row_tower : per_row_conv) * rows[i];
            }
            a.tower_flop += per_row_tower * rows[i];
        }
    }
    return 0;
}

// game g's history: start[g] (startpos when start is NULL), then hist[off[g]..off[g+1]) played;
// the root is the last position, the earlier ones are its repetition history (pos_count, chess.rs:16)
int upload_histories(az_search* s, const az_pos* start, const int32_t* hist, const int32_t* off,
                     const int32_t* game_id, const int32_t* noise_ply) {
    const int G = s->E.G;
    std::vector<azc::Pos> hp((size_t)G * HMAX);
    std::vector<int> hl(G), gids(G), plies(G), act(G, 1);
    for (int g = 0; g < G; g++) {
        azc::Pos p = azc::startpos();
        if (start) {
            p = *reinterpret_cast<const azc::Pos*>(start + g);
            if (const char* why = azc::setup_error(p))   // before finalize: its generator assumes one king per side
                return fail("root start position of game " + std::to_string(g) + " rejected: " + why);
            bool chk;
            azc::finalize(p, &chk);          // flags / rep_key from the position itself
        }
        std::vector<azc::Pos> H{p};
        const int b = off ? off[g] : 0, e = off ? off[g + 1] : 0;
        for (int i = b; i < e; i++) {
            int32_t lst[AZ_MAX_MOVES];
            const int nl = az_pos_legal_indices(reinterpret_cast<const az_pos*>(&p), lst, AZ_MAX_MOVES);
            bool ok = false;
            for (int k = 0; k < nl; k++) ok |= lst[k] == hist[i];
            if (!ok) return fail("illegal move in root history of game " + std::to_string(g));
            p = azc::play_index(p, hist[i]);
            bool chk;
            azc::finalize(p, &chk);
            H.push_back(p);
        }
        if ((int)H.size() > HMAX) return fail("history too long");
        bool chk;
        azc::Pos q = p;
        if (azc::finalize(q, &chk) == 0) return fail("root of game " + std::to_string(g) + " has no legal move");
        for (size_t i = 0; i < H.size(); i++) hp[(size_t)g * HMAX + i] = H[i];
        hl[g] = (int)H.size();
        gids[g] = game_id ? game_id[g] : g;
        plies[g] = noise_ply ? noise_ply[g] : (e - b);
    }
    Engine& E = s->E;
    AZ_HIP(hipMemcpy(E.hist, hp.data(), hp.size() * sizeof(azc::Pos), hipMemcpyHostToDevice));
    AZ_HIP(hipMemcpy(E.hist_len, hl.data(), G * 4, hipMemcpyHostToDevice));
    AZ_HIP(hipMemcpy(E.game_id, gids.data(), G * 4, hipMemcpyHostToDevice));
    AZ_HIP(hipMemcpy(E.ply, plies.data(), G * 4, hipMemcpyHostToDevice));
    AZ_HIP(hipMemcpy(E.active, act.data(), G * 4, hipMemcpyHostToDevice));
    return 0;
}

int setup_roots(az_search* s, int apply_noise, bool save_template) {
    Engine& E = s->E;
    s->sim_cursor = 0;                 // new roots abandon any self-play move in progress
    AZ_HIP(hipMemsetAsync(E.ctr->batch_count, 0, sizeof(E.ctr->batch_count), s->st));
    k_root_setup<<<(E.G + 63) / 64, 64, 0, s->st>>>(E);
    int rc = eval_rows(s);
    if (rc) return rc;
    AZ_HIP(hipMemsetAsync(E.ctr->batch_count, 0, sizeof(int), s->st));   // simulation step 0 allocates from [0]
    if (save_template) k_save_start_template<<<1, 256, 0, s->st>>>(E);
    k_root_noise<<<E.G, 64, 0, s->st>>>(E, apply_noise);
    AZ_HIP(hipGetLastError());
    AZ_HIP(hipStreamSynchronize(s->st));
    return 0;
}

int drain_records(az_search* s) {
    Counters c;
    AZ_HIP(hipMemcpyAsync(&c, s->E.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s->st));
    AZ_HIP(hipStreamSynchronize(s->st));
    int nrec = std::min(c.rec_count, s->E.rec_cap);
    if (c.rec_count > s->E.rec_cap) return fail("step record buffer overflow");
    if (nrec == 0) return 0;
    std::vector<StepRec> recs(nrec);
    AZ_HIP(hipMemcpy(recs.data(), s->E.recs, (size_t)nrec * sizeof(StepRec), hipMemcpyDeviceToHost));
    AZ_HIP(hipMemsetAsync(&s->E.ctr->rec_count, 0, sizeof(int), s->st));
    // keep device order per game: steps were appended in ply order within a game
    std::stable_sort(recs.begin(), recs.end(), [](const StepRec& a, const StepRec& b) {
        return a.game_id != b.game_id ? a.game_id < b.game_id : (a.kind != b.kind ? a.kind < b.kind : a.ply < b.ply);
    });
    for (const StepRec& r : recs) {
        if (r.kind == 0) { s->pending[r.game_id].push_back(r); continue; }
        auto it = s->pending.find(r.game_id);
        if (it == s->pending.end()) continue;
        // final value = turn * result * (1 - fullmoves / (2 * NUM_FULLMOVES))  (training.rs:332-335)
        const float result = r.result == azc::WHITE_WINS ? 1.0f : (r.result == azc::BLACK_WINS ? -1.0f : 0.0f);
        const float decay = 1.0f - ((float)r.end_fullmoves / (2.0f * (float)azc::NUM_FULLMOVES));
        for (const StepRec& st : it->second) {
            az_episode_step o;
            memset(&o, 0, sizeof(o));
            const float turn = st.pos.turn == 0 ? 1.0f : -1.0f;
            o.game_id = st.game_id; o.ply = st.ply; o.action = st.action; o.search_depth = st.depth;
            o.final_value = turn * (result * decay);
            o.result = r.result;
            o.nvis = st.nvis;
            memcpy(&o.state, &st.pos, sizeof(az_pos));
            memcpy(o.vis_idx, st.vis_idx, sizeof(o.vis_idx));
            memcpy(o.vis_n, st.vis_n, sizeof(o.vis_n));
            s->finished.push_back(o);
        }
        s->pending.erase(it);
    }
    return 0;
}

}  // namespace

extern "C" {

int az_search_default_cfg(az_search_cfg* c) {
    if (!c) return fail("null cfg");
    memset(c, 0, sizeof(*c));
    c->games = 100;          // NUM_EPISODES parameters.rs:13
    c->sims = 256;           // NUM_SIMULATIONS parameters.rs:32
    c->c_puct = 3.0f;        // parameters.rs:34
    c->dir_alpha = 0.3f;     // parameters.rs:28
    c->dir_eps = 0.25f;      // parameters.rs:29
    c->temp_moves = 15;      // parameters.rs:31
    c->noise = 1;
    c->seed = 42;            // parameters.rs:6
    c->evaluator = AZ_EVAL_NET;
    c->continuous = 0;
    c->record_evals = 0;
    c->eval_log_cap = 0;
    c->cache_capacity = 500000;   // CACHE_CAPACITY parameters.rs:4
    return 0;
}

int az_search_create(az_net* net, const az_search_cfg* cfg, int device, az_search** out) {
    if (!cfg || !out) return fail("null argument");
    if (cfg->games <= 0 || cfg->sims <= 0 || cfg->sims > 60000) return fail("bad games/sims");
    if (cfg->evaluator != AZ_EVAL_NET && cfg->evaluator != AZ_EVAL_SYNTHETIC && cfg->evaluator != AZ_EVAL_CALLBACK)
        return fail("bad evaluator (AZ_EVAL_NET / AZ_EVAL_SYNTHETIC / AZ_EVAL_CALLBACK)");
    if (cfg->evaluator == AZ_EVAL_NET && !net) return fail("AZ_EVAL_NET needs a network");
    AZ_HIP(hipSetDevice(device));
    az_search* s = new az_search();
    s->cfg = *cfg;
    s->device = device;
    s->net = net;
    if (const char* v = getenv("AZ_FUSED_STEPS")) s->fused_steps = atoi(v) != 0;   // A/B and parity tests
    if (const char* v = getenv("AZ_PERSIST")) s->persist = atoi(v);
    AZ_HIP(hipDeviceGetAttribute(&s->cus, hipDeviceAttributeMultiprocessorCount, device));
    AZ_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    Engine& E = s->E;
    const int G = cfg->games, S = cfg->sims;
    E.G = G; E.S = S; E.NMAX = S + 2; E.PMAX = S + 2;
    E.EMAX = E.NMAX * 218 + MAX_EDGES;
    // sims <= 60000 (checked above) keeps EMAX < 2^24: child_hdr packs edge_begin in 24 bits
    E.c_puct = cfg->c_puct; E.dir_alpha = cfg->dir_alpha; E.dir_eps = cfg->dir_eps;
    E.temp_moves = cfg->temp_moves; E.noise = cfg->noise; E.continuous = cfg->continuous; E.seed = cfg->seed;
    int rc = 0;
    rc |= dalloc(s, &E.nodes, (size_t)G * E.NMAX);
    rc |= dalloc(s, &E.npos, (size_t)G * E.NMAX);
    rc |= dalloc(s, &E.edges, (size_t)G * E.EMAX);
    rc |= dalloc(s, &E.child_hdr, (size_t)G * E.EMAX);
    rc |= dalloc(s, &E.node_count, G); rc |= dalloc(s, &E.edge_count, G); rc |= dalloc(s, &E.max_depth, G);
    rc |= dalloc(s, &E.leaf_node, G); rc |= dalloc(s, &E.leaf_edge, G); rc |= dalloc(s, &E.leaf_len, G);
    rc |= dalloc(s, &E.leaf_kind, G); rc |= dalloc(s, &E.leaf_row, G);
    rc |= dalloc(s, &E.path_node, (size_t)G * E.PMAX); rc |= dalloc(s, &E.path_edge, (size_t)G * E.PMAX);
    rc |= dalloc(s, &E.hist, (size_t)G * HMAX); rc |= dalloc(s, &E.hist_len, G);
    rc |= dalloc(s, &E.game_id, G); rc |= dalloc(s, &E.ply, G); rc |= dalloc(s, &E.active, G);
    rc |= dalloc(s, &E.row_game, G); rc |= dalloc(s, &E.row_node, G); rc |= dalloc(s, &E.value, G);
    float* sq = nullptr;
    rc |= dalloc(s, &sq, S + 2);
    rc |= dalloc(s, &E.start_edges, MAX_EDGES); rc |= dalloc(s, &E.start_n, 1);
    E.rec_cap = 2 * G + 16;
    rc |= dalloc(s, &E.recs, E.rec_cap);
    rc |= dalloc(s, &E.ctr, 1);
    rc |= dalloc(s, &E.batch_hist, S);
    rc |= dalloc(s, &E.cached_value, G);
    rc |= dalloc(s, &E.g_sims, G); rc |= dalloc(s, &E.g_sel_bytes, G); rc |= dalloc(s, &E.g_evals, G);
#ifdef AZ_STEP_TRACE
    rc |= dalloc(s, &E.trace, (size_t)G * 16);
#endif
    E.cache_mask = -1;
    if (cfg->cache_capacity > 0) {
        int slots = 1;
        while (slots < cfg->cache_capacity) slots <<= 1;
        E.cache_mask = slots - 1;
        rc |= dalloc(s, &E.c_state, slots); rc |= dalloc(s, &E.c_key, slots); rc |= dalloc(s, &E.c_pos, slots);
        rc |= dalloc(s, &E.c_value, slots); rc |= dalloc(s, &E.c_n, slots);
        rc |= dalloc(s, &E.c_pri, (size_t)slots * MAX_EDGES);
    }
    if (rc) { az_search_destroy(s); return -1; }
    std::vector<float> st(S + 2);
    for (int i = 0; i < S + 2; i++) st[i] = sqrtf((float)i);    // f32 sqrt, correctly rounded
    AZ_HIP(hipMemcpy(sq, st.data(), st.size() * 4, hipMemcpyHostToDevice));
    E.sqrt_tab = sq;
    if (cfg->record_evals) {
        E.log_cap = cfg->eval_log_cap > 0 ? cfg->eval_log_cap : 1 << 16;
        E.log_prior_cap = E.log_cap * 64;
        rc |= dalloc(s, &E.log_key, E.log_cap); rc |= dalloc(s, &E.log_value, E.log_cap);
        rc |= dalloc(s, &E.log_off, E.log_cap); rc |= dalloc(s, &E.log_n, E.log_cap);
        rc |= dalloc(s, &E.log_idx, E.log_prior_cap); rc |= dalloc(s, &E.log_prior, E.log_prior_cap);
        if (rc) { az_search_destroy(s); return -1; }
    }
    if (cfg->evaluator == AZ_EVAL_NET) {
        const NetDev* n = net->dev;
        if (n->device != device) { az_search_destroy(s); return fail("net and search on different devices"); }
        const size_t ab = act_bytes(n->dtype);
        char* p = nullptr;
        rc |= dalloc(s, &p, (size_t)G * 64 * 32 * ab); s->planes = p;
        rc |= dalloc(s, &p, (size_t)G * 64 * n->filters * ab); s->x = p;
        rc |= dalloc(s, &p, (size_t)G * 64 * n->filters * ab); s->h = p;
        if (rc) { az_search_destroy(s); return -1; }
    }
    if (cfg->evaluator == AZ_EVAL_CALLBACK) {
        rc |= dalloc(s, &s->d_pos, G); rc |= dalloc(s, &s->d_pol, (size_t)G * AZ_ACTION_SPACE); rc |= dalloc(s, &s->d_val, G);
        if (!rc && (hipHostMalloc((void**)&s->h_pos, (size_t)G * sizeof(azc::Pos)) != hipSuccess ||
                    hipHostMalloc((void**)&s->h_pol, (size_t)G * AZ_ACTION_SPACE * 4) != hipSuccess ||
                    hipHostMalloc((void**)&s->h_val, (size_t)G * 4) != hipSuccess))
            rc = fail("hipHostMalloc failed (evaluator staging)");
        if (rc) { az_search_destroy(s); return -1; }
    }
    SearchOut& so = s->so;
    so.nodes = E.nodes; so.edges = E.edges; so.NMAX = E.NMAX; so.EMAX = E.EMAX;
    so.row_game = E.row_game; so.row_node = E.row_node; so.value = E.value;
    so.log_cap = E.log_cap; so.log_prior_cap = E.log_prior_cap;
    so.log_key = E.log_key; so.log_value = E.log_value; so.log_off = E.log_off; so.log_n = E.log_n;
    so.log_idx = E.log_idx; so.log_prior = E.log_prior; so.ctr = E.ctr; so.npos = E.npos;
    *out = s;
    return 0;
}

int az_search_destroy(az_search* s) {
    if (!s) return 0;
    (void)hipSetDevice(s->device);
    if (s->st) (void)hipStreamSynchronize(s->st);
    for (void* p : s->allocs) (void)hipFree(p);
    for (void* p : {(void*)s->h_pos, (void*)s->h_pol, (void*)s->h_val})
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : s->ev) (void)hipEventDestroy(e);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    return 0;
}

int az_search_set_evaluator(az_search* s, az_eval_fn fn, void* ctx) {
    if (!s || !fn) return fail("null argument");
    if (s->cfg.evaluator != AZ_EVAL_CALLBACK) return fail("az_search_set_evaluator: cfg.evaluator is not AZ_EVAL_CALLBACK");
    s->eval_fn = fn;
    s->eval_ctx = ctx;
    return 0;
}

int az_search_set_roots(az_search* s, const int32_t* hist, const int32_t* off, const int32_t* game_id,
                        const int32_t* noise_ply, int apply_noise) {
    return az_search_set_roots_from(s, nullptr, hist, off, game_id, noise_ply, apply_noise);
}

int az_search_set_roots_from(az_search* s, const az_pos* start, const int32_t* hist, const int32_t* off,
                             const int32_t* game_id, const int32_t* noise_ply, int apply_noise) {
    if (!s) return fail("null search");
    AZ_HIP(hipSetDevice(s->device));
    int rc = upload_histories(s, start, hist, off, game_id, noise_ply);
    if (rc) return rc;
    rc = setup_roots(s, apply_noise, false);
    s->roots_fresh = rc == 0;
    return rc;
}

static int read_roots(az_search* s, float* improved, uint32_t* visits, int32_t* depth) {
    const int G = s->E.G;
    float* di = nullptr; uint32_t* dv = nullptr; int* dd = nullptr;
    if (improved) AZ_HIP(hipMalloc(&di, (size_t)G * AZ_ACTION_SPACE * 4));
    if (visits) AZ_HIP(hipMalloc(&dv, (size_t)G * AZ_ACTION_SPACE * 4));
    if (depth) AZ_HIP(hipMalloc(&dd, (size_t)G * 4));
    k_readout<<<G, 256, 0, s->st>>>(s->E, di, dv, dd);
    AZ_HIP(hipGetLastError());
    if (improved) AZ_HIP(hipMemcpyAsync(improved, di, (size_t)G * AZ_ACTION_SPACE * 4, hipMemcpyDeviceToHost, s->st));
    if (visits) AZ_HIP(hipMemcpyAsync(visits, dv, (size_t)G * AZ_ACTION_SPACE * 4, hipMemcpyDeviceToHost, s->st));
    if (depth) AZ_HIP(hipMemcpyAsync(depth, dd, (size_t)G * 4, hipMemcpyDeviceToHost, s->st));
    AZ_HIP(hipStreamSynchronize(s->st));
    (void)hipFree(di); (void)hipFree(dv); (void)hipFree(dd);
    return 0;
}

int az_search_run(az_search* s, float* improved, uint32_t* visits, int32_t* depth) {
    if (!s) return fail("null search");
    if (!s->roots_fresh) return fail("az_search_run: set roots (az_search_set_roots / az_search_advance) first");
    s->roots_fresh = false;
    AZ_HIP(hipSetDevice(s->device));
    int rc = run_sims(s);
    if (rc) return rc;
    return read_roots(s, improved, visits, depth);
}

int az_search_read_roots(az_search* s, float* improved, uint32_t* visits, int32_t* depth) {
    if (!s) return fail("null search");
    AZ_HIP(hipSetDevice(s->device));
    return read_roots(s, improved, visits, depth);
}

int az_search_advance(az_search* s, const int32_t* actions, int apply_noise, int32_t* result) {
    if (!s || !actions) return fail("null argument");
    AZ_HIP(hipSetDevice(s->device));
    const int G = s->E.G;
    int *da = nullptr, *dr = nullptr;
    AZ_HIP(hipMalloc(&da, G * 4));
    AZ_HIP(hipMalloc(&dr, G * 4));
    std::vector<int> init(G, azc::ILLEGAL);
    AZ_HIP(hipMemcpy(dr, init.data(), G * 4, hipMemcpyHostToDevice));
    AZ_HIP(hipMemcpy(da, actions, G * 4, hipMemcpyHostToDevice));
    k_finish<<<G, 64, 0, s->st>>>(s->E, 1, da, dr, apply_noise);
    AZ_HIP(hipGetLastError());
    AZ_HIP(hipStreamSynchronize(s->st));
    std::vector<int> res(G);
    AZ_HIP(hipMemcpy(res.data(), dr, G * 4, hipMemcpyDeviceToHost));
    (void)hipFree(da); (void)hipFree(dr);
    s->roots_fresh = true;
    s->sim_cursor = 0;                 // re-rooted: a self-play move in progress is abandoned
    if (result) memcpy(result, res.data(), G * 4);
    return 0;
}

int az_selfplay_reset(az_search* s) {
    if (!s) return fail("null search");
    AZ_HIP(hipSetDevice(s->device));
    int rc = upload_histories(s, nullptr, nullptr, nullptr, nullptr, nullptr);
    if (rc) return rc;
    AZ_HIP(hipMemset(s->E.ctr, 0, sizeof(Counters)));
    AZ_HIP(hipMemset(s->E.g_sims, 0, (size_t)s->E.G * 8));
    AZ_HIP(hipMemset(s->E.g_evals, 0, (size_t)s->E.G * 8));
    if (s->E.cache_mask >= 0) AZ_HIP(hipMemset(s->E.c_state, 0, (size_t)(s->E.cache_mask + 1) * sizeof(unsigned)));
    const int G = s->E.G;
    AZ_HIP(hipMemcpy(&s->E.ctr->next_game_id, &G, 4, hipMemcpyHostToDevice));
    s->pending.clear();
    s->finished.clear();
    s->finished_read = 0;
    s->sim_cursor = 0;
    return setup_roots(s, s->cfg.noise, true);
}

static int selfplay_sims(az_search* s, int nsims, int* finished, int* active, int* move_done) {
    if (!s) return fail("null search");
    if (nsims <= 0) return fail("az_selfplay_run_sims: nsims must be > 0");
    AZ_HIP(hipSetDevice(s->device));
    unsigned long long before = 0;
    AZ_HIP(hipMemcpy(&before, &s->E.ctr->games_finished, 8, hipMemcpyDeviceToHost));
    const int i0 = s->sim_cursor, i1 = std::min(s->E.S, i0 + nsims);
    int rc = run_sims(s, i0, i1);
    if (rc) return rc;
    s->sim_cursor = i1;
    if (move_done) *move_done = i1 == s->E.S;
    if (i1 < s->E.S) {                 // the move is not complete: no action yet
        if (finished) *finished = 0;
        if (active) *active = -1;
        return 0;
    }
    s->sim_cursor = 0;
    k_finish<<<s->E.G, 64, 0, s->st>>>(s->E, 0, nullptr, nullptr, s->cfg.noise);
    AZ_HIP(hipGetLastError());
    rc = drain_records(s);
    if (rc) return rc;
    unsigned long long after = 0;
    AZ_HIP(hipMemcpy(&after, &s->E.ctr->games_finished, 8, hipMemcpyDeviceToHost));
    if (finished) *finished = (int)(after - before);
    if (active) {
        std::vector<int> a(s->E.G);
        AZ_HIP(hipMemcpy(a.data(), s->E.active, s->E.G * 4, hipMemcpyDeviceToHost));
        int n = 0;
        for (int v : a) n += v != 0;
        *active = n;
    }
    return 0;
}

int az_selfplay_step(az_search* s, int* finished, int* active) {
    if (s && s->sim_cursor != 0) return fail("az_selfplay_step: a move is in progress (az_selfplay_run_sims)");
    return selfplay_sims(s, s ? s->E.S : 1, finished, active, nullptr);
}

int az_selfplay_run_sims(az_search* s, int nsims, int* finished, int* active, int* move_done) {
    return selfplay_sims(s, nsims, finished, active, move_done);
}

int az_selfplay_drain(az_search* s, az_episode_step* out, int cap) {
    if (!s) return fail("null search");
    int n = 0;
    while (s->finished_read < s->finished.size() && n < cap) {
        if (out) out[n] = s->finished[s->finished_read];
        n++;
        s->finished_read++;
    }
    if (s->finished_read == s->finished.size()) { s->finished.clear(); s->finished_read = 0; }
    return n;
}

int az_search_persistent(az_search* s) { return s && use_persistent(s) ? 1 : 0; }

int az_search_stats_get(az_search* s, az_search_stats* out) {
    if (!s || !out) return fail("null argument");
    AZ_HIP(hipSetDevice(s->device));
    AZ_HIP(hipStreamSynchronize(s->st));
    Counters c;
    AZ_HIP(hipMemcpy(&c, s->E.ctr, sizeof(c), hipMemcpyDeviceToHost));
    out->sims = (int64_t)(c.sims + sum_games(s, s->E.g_sims));
    const unsigned long long ge = sum_games(s, s->E.g_evals);
    out->evals = (int64_t)(c.evals + ge);
    out->terminal_leaves = (int64_t)c.terminal;
    out->games_finished = (int64_t)c.games_finished;
    out->moves = (int64_t)c.moves;
    out->max_depth_sum = (int64_t)c.depth_sum;
    out->cache_hits = (int64_t)c.cache_hits;
    out->cache_misses = (int64_t)(c.evals + ge);
    out->overflow = c.overflow;
    std::vector<int> nc(s->E.G), ec(s->E.G);
    AZ_HIP(hipMemcpy(nc.data(), s->E.node_count, s->E.G * 4, hipMemcpyDeviceToHost));
    AZ_HIP(hipMemcpy(ec.data(), s->E.edge_count, s->E.G * 4, hipMemcpyDeviceToHost));
    out->max_nodes = *std::max_element(nc.begin(), nc.end());
    out->max_edges = *std::max_element(ec.begin(), ec.end());
    out->node_cap = s->E.NMAX;
    out->edge_cap = s->E.EMAX;
    return 0;
}

int az_search_eval_log(az_search* s, int64_t* n_rows, int64_t* n_priors, uint64_t* keys, float* values,
                       int32_t* off, int32_t* idx, float* priors) {
    if (!s) return fail("null search");
    AZ_HIP(hipSetDevice(s->device));
    AZ_HIP(hipStreamSynchronize(s->st));
    Counters c;
    AZ_HIP(hipMemcpy(&c, s->E.ctr, sizeof(c), hipMemcpyDeviceToHost));
    if (c.log_count > s->E.log_cap || c.log_prior_count > s->E.log_prior_cap) return fail("eval log overflow");
    const int nr = c.log_count;
    if (n_rows) *n_rows = nr;
    if (n_priors) *n_priors = c.log_prior_count;
    if (!keys) return 0;
    std::vector<int> o(nr), nn(nr);
    AZ_HIP(hipMemcpy(keys, s->E.log_key, (size_t)nr * 8, hipMemcpyDeviceToHost));
    AZ_HIP(hipMemcpy(values, s->E.log_value, (size_t)nr * 4, hipMemcpyDeviceToHost));
    AZ_HIP(hipMemcpy(o.data(), s->E.log_off, (size_t)nr * 4, hipMemcpyDeviceToHost));
    AZ_HIP(hipMemcpy(nn.data(), s->E.log_n, (size_t)nr * 4, hipMemcpyDeviceToHost));
    std::vector<int> di(c.log_prior_count);
    std::vector<float> dp(c.log_prior_count);
    AZ_HIP(hipMemcpy(di.data(), s->E.log_idx, di.size() * 4, hipMemcpyDeviceToHost));
    AZ_HIP(hipMemcpy(dp.data(), s->E.log_prior, dp.size() * 4, hipMemcpyDeviceToHost));
    // compact to CSR in row order
    int64_t pos = 0;
    for (int r = 0; r < nr; r++) {
        off[r] = (int32_t)pos;
        for (int k = 0; k < nn[r]; k++) { idx[pos] = di[o[r] + k]; priors[pos] = dp[o[r] + k]; pos++; }
    }
    off[nr] = (int32_t)pos;
    return 0;
}

int az_search_timing(az_search* s, az_timing* out, int reset, int enable) {
    if (!s) return fail("null search");
    AZ_HIP(hipSetDevice(s->device));
    if (out) {
        *out = s->acc;
        AZ_HIP(hipStreamSynchronize(s->st));
        out->select_bytes = (double)sum_games(s, s->E.g_sel_bytes);
    }
    if (reset) {
        s->acc = az_timing{};
        AZ_HIP(hipMemset(s->E.g_sel_bytes, 0, (size_t)s->E.G * 8));
    }
    s->timing = enable != 0;
    return 0;
}

}  // extern "C"

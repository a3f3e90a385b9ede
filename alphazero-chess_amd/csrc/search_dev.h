// search_dev.h -- device side of the GPU tree search (tree.rs select / expand / backup), shared by
// search.hip (the per-step kernels) and tower.hip (the persistent per-game simulation kernel,
// k_sims32w, which runs a game's tree steps and its network evaluations in one workgroup).
// Everything here is __device__ __forceinline__ (or constexpr), so each translation unit gets its
// own copy and no kernel symbol is defined twice.
#pragma once
#include "az_internal.h"
#include "detmath.h"

#pragma clang fp contract(off)

namespace azi {
__device__ __forceinline__ Node* game_nodes(const Engine& E, int g) { return E.nodes + (size_t)g * E.NMAX; }
__device__ __forceinline__ Edge* game_edges(const Engine& E, int g) { return E.edges + (size_t)g * E.EMAX; }
__device__ __forceinline__ azc::Pos* game_npos(const Engine& E, int g) { return E.npos + (size_t)g * E.NMAX; }

__device__ __forceinline__ int* step_rows(const Engine& E, int step) { return &E.ctr->batch_count[step & 1]; }

// ------------------------------------------------------------------ wave primitives (DPP / ballot)
// Cross-lane reductions without LDS: __shfl_* lower to ds_bpermute (~100+ cycles a step on a lone
// wave), DPP moves run at VALU latency.  gfx9 row_bcast15/31 carry row maxima across the 4 rows.
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ float dpp_f32(float old, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                 __builtin_bit_cast(int, v), CTRL, ROWMASK, 0xF, false));
}
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ int dpp_i32(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xF, false);
}
// maximum over the wave of a non-NaN float (all lanes active); result wave-uniform
__device__ __forceinline__ float wave_max_f32(float v) {
    v = fmaxf(v, dpp_f32<0xB1>(v, v));         // quad_perm [1,0,3,2]
    v = fmaxf(v, dpp_f32<0x4E>(v, v));         // quad_perm [2,3,0,1]
    v = fmaxf(v, dpp_f32<0x141>(v, v));        // row_half_mirror
    v = fmaxf(v, dpp_f32<0x140>(v, v));        // row_mirror: every lane holds its row's max
    v = fmaxf(v, dpp_f32<0x142, 0xA>(v, v));   // row_bcast:15 -> rows 1, 3
    v = fmaxf(v, dpp_f32<0x143, 0xC>(v, v));   // row_bcast:31 -> rows 2, 3: lane 63 = wave max
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ int wave_min_i32(int v) {
    v = min(v, dpp_i32<0xB1>(v, v));
    v = min(v, dpp_i32<0x4E>(v, v));
    v = min(v, dpp_i32<0x141>(v, v));
    v = min(v, dpp_i32<0x140>(v, v));
    v = min(v, dpp_i32<0x142, 0xA>(v, v));
    v = min(v, dpp_i32<0x143, 0xC>(v, v));
    return __builtin_amdgcn_readlane(v, 63);
}
// sum over the wave (all lanes active); result wave-uniform.  Lanes outside a row_bcast's row
// mask keep `old` = 0, so nothing is counted twice.
__device__ __forceinline__ int wave_sum_i32(int v) {
    v += dpp_i32<0xB1>(0, v);
    v += dpp_i32<0x4E>(0, v);
    v += dpp_i32<0x141>(0, v);
    v += dpp_i32<0x140>(0, v);
    v += dpp_i32<0x142, 0xA>(0, v);
    v += dpp_i32<0x143, 0xC>(0, v);
    return __builtin_amdgcn_readlane(v, 63);
}
// exclusive prefix sum over the wave of a small count (0..31) by its bits: one ballot and one
// mbcnt per bit; *total = the wave sum (uniform)
__device__ __forceinline__ int wave_excl_small(int cnt, int* total) {
    int pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) {
        const unsigned long long m = __ballot((cnt >> b) & 1);
        pre += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
        tot += __popcll(m) << b;
    }
    *total = tot;
    return pre;
}

// ------------------------------------------------------------------ select
// one wavefront walks game g (active) from the root to a leaf
__device__ __forceinline__ void select_game(const Engine& E, int g, int lane) {
    const Node* nodes = game_nodes(E, g);
    const Edge* edges = game_edges(E, g);
    int* pn = E.path_node + (size_t)g * E.PMAX;
    int* pe = E.path_edge + (size_t)g * E.PMAX;
    const float cp = E.c_puct;
    const uint32_t* chdr = E.child_hdr + (size_t)g * E.EMAX;
    int node = 0, len = 0;
    unsigned long long bytes = 0;
    // the current node's edge range: the root's from its record; below it, from the child_hdr
    // entry of the edge that leads there, read together with that edge -- one dependent load
    // round per level.  Nt - 1 = sum of the node's edge visits (= its nsum: every backup adds one
    // to both), summed on DPP from the edges already loaded.
    const Node rt = nodes[0];
    int ebeg = (int)rt.edge_begin, nedg = rt.nedges;
    for (;;) {
        float best = -INFINITY;
        int bpos = 0x7fffffff, bchild = CHILD_NONE;
        uint32_t bhdr = 0u;
        if (nedg <= 64) {
            const int e = min(lane, nedg - 1);             // unconditional (clamped) loads
            const Edge ed = edges[ebeg + e];
            const uint32_t hd = chdr[ebeg + e];
            const int nsum = wave_sum_i32(lane < nedg ? (int)ed.N : 0);
            // sqrt(Nt) in-line (IEEE correctly rounded, as the host's sqrtf in the oracle)
            const float sq = sqrtf((float)(nsum + 1));
            const float Nf = (float)ed.N;
            const float u = cp * ed.P * sq / (1.0f + Nf);
            const float q = ed.N > 0 ? ed.W / Nf : 0.0f;
            const float v = q + u;
            if (lane < nedg && v > best) { best = v; bpos = lane; bchild = ed.child; bhdr = hd; }
        } else {
            const float sq = sqrtf((float)(nodes[node].nsum + 1));
            for (int e = lane; e < nedg; e += 64) {
                const Edge ed = edges[ebeg + e];
                const uint32_t hd = chdr[ebeg + e];
                const float Nf = (float)ed.N;
                const float u = cp * ed.P * sq / (1.0f + Nf);
                const float q = ed.N > 0 ? ed.W / Nf : 0.0f;
                const float v = q + u;
                if (v > best) { best = v; bpos = e; bchild = ed.child; bhdr = hd; }
            }
        }
        // wave argmax, first maximum in `moves` order: the wave max, then the lowest edge index
        // among the lanes holding it (lane order = edge order while nedges <= 64); the winner's
        // child id and child header come from the records that lane already holds
        int child;
        uint32_t hdr;
        {
            const float wmax = wave_max_f32(best);
            const unsigned long long hit = __ballot(best == wmax);
            int wl;
            if (nedg <= 64) {
                wl = (int)__builtin_ctzll(hit);
                bpos = __builtin_amdgcn_readlane(bpos, wl);
            } else {
                const int mn = wave_min_i32(best == wmax ? bpos : 0x7fffffff);
                wl = (int)__builtin_ctzll(__ballot(best == wmax && bpos == mn));
                bpos = mn;
            }
            child = __builtin_amdgcn_readlane(bchild, wl);
            hdr = (uint32_t)__builtin_amdgcn_readlane((int)bhdr, wl);
        }
        bytes += 20ull * nedg;
        // no edge beat -inf: every value is NaN (a diverged network).  The reference keeps its
        // initial idx (tree.rs:121-131); the engine takes the first edge instead of reading
        // past the node's edge list.
        if (bpos >= nedg) {
            bpos = 0;
            child = edges[ebeg].child;
            hdr = chdr[ebeg];
        }
        const int eabs = ebeg + bpos;
        if (lane == 0) { pn[len] = node; pe[len] = eabs; }
        len++;
        if (child >= 0 && len < E.PMAX) {
            node = child;
            ebeg = (int)(hdr >> 8);
            nedg = (int)(hdr & 255u);
            continue;
        }
        if (lane == 0) {
            E.leaf_node[g] = node;
            E.leaf_edge[g] = eabs;
            E.leaf_len[g] = len;
            E.leaf_kind[g] = child == CHILD_DRAW ? LEAF_DRAW : (child == CHILD_WIN ? LEAF_WIN : LEAF_EVAL);
            E.g_sel_bytes[g] += bytes;   // per-game slot: no same-address atomic across 2048 waves
        }
        return;
    }
}


// ------------------------------------------------------------------ FEN cache
constexpr int CACHE_PROBES = 4;

__device__ __forceinline__ bool same_fen(const azc::Pos& a, const azc::Pos& b) {   // FEN(PseudoLegal) equality
    for (int i = 0; i < 8; i++) if (a.bb[i] != b.bb[i]) return false;
    return a.turn == b.turn && a.castling == b.castling && a.ep == b.ep && a.halfmoves == b.halfmoves &&
           a.fullmoves == b.fullmoves;
}


// ------------------------------------------------------------------ expand
struct EdgeSink {
    Edge* out;
    int n;
    __device__ void operator()(int idx) {
        Edge e;
        e.P = 0.0f; e.W = 0.0f; e.N = 0; e.idx = (uint16_t)idx; e.child = CHILD_NONE;
        out[n++] = e;
    }
};

enum { X_NONE = 0, X_ROW, X_TERMINAL, X_CACHED };

// ------------------------------------------------------------------ wave-parallel expansion
// One game's expansion with the 64 lanes of a wavefront: the legal-move list of the new leaf in
// shakmaty order (azc::gen_legal's order), generated by square -- lane s owns
// square s (the from-square; the to-square for pawn pushes) -- with one wave prefix sum per
// generation group giving every move its position; the repetition count compares one earlier
// position per lane.  Every value a branch depends on is wave-uniform.
// move_to_index (chess.rs:73-116, azc::move_index) as selects only: the lanes of a wave index
// different moves at once, and the if-chain form diverges into up to 12 serial paths
__device__ __forceinline__ int move_index_bf(int from, int to, int turn) {
    const int file = from & 7, rank = turn ? 7 - (from >> 3) : (from >> 3);
    const int dfile = to & 7, drank = turn ? 7 - (to >> 3) : (to >> 3);
    const int df = dfile - file, dr = drank - rank;
    const int adf = df < 0 ? -df : df;
    const int kn = df > 0 ? (dr > 0 ? (adf == 1 ? 0 : 1) : (adf == 2 ? 2 : 3))
                          : (dr < 0 ? (adf == 1 ? 4 : 5) : (adf == 2 ? 6 : 7));
    const int qp = df == 0 ? (dr > 0 ? 7 + dr : 35 - dr)
                 : dr == 0 ? (df > 0 ? 21 + df : 49 - df)
                 : df > 0 ? (dr > 0 ? 14 + dr : 28 + df) : (dr < 0 ? 42 - dr : 56 - df);
    const int plane = df != 0 && dr != 0 && adf + (dr < 0 ? -dr : dr) == 3 ? kn : qp;
    return plane * 64 + rank * 8 + file;
}

constexpr int GEN_WAVES = 4;   // waves per workgroup that may run gen_legal_wave (k_step STEP_WPB <= 4)
// NW: waves of the workgroup that run it (the LDS staging rows it reserves; k_sims32w: wave 0 only)
template <int NW = GEN_WAVES>
__device__ __forceinline__ int gen_legal_wave(const azc::Pos& p, Edge* __restrict__ out, int lane, bool* in_check,
                                           bool* legal_ep, unsigned long long* tr = nullptr) {
    using namespace azc;
    const int us = p.turn, them = us ^ 1;
    const uint64_t our = side_bb(p, us), their = side_bb(p, them);
    const uint64_t occ = our | their, empty = ~occ;
    const uint64_t kbb = p.bb[KING] & our;
    const int ksq = ctz64(kbb);
    const uint64_t tP = p.bb[PAWN] & their, tN = p.bb[KNIGHT] & their, tK = p.bb[KING] & their;
    const uint64_t tB = (p.bb[BISHOP] | p.bb[QUEEN]) & their, tR = (p.bb[ROOK] | p.bb[QUEEN]) & their;
    const uint64_t checkers = (pawn_att(us, kbb) & tP) | (knight_att(kbb) & tN) | (bishop_att(kbb, empty) & tB) |
                              (rook_att(kbb, empty) & tR);
    const uint64_t empty_xk = empty | kbb;
    const uint64_t attacked = pawn_att(them, tP) | knight_att(tN) | king_att(tK) | bishop_att(tB, empty_xk) |
                              rook_att(tR, empty_xk);
    uint64_t pinned = 0, pinray[8], checkmask = checkers;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        const uint64_t r = ray_dir(d, kbb, empty);
        const uint64_t sl = (d & 1) ? tB : tR;
        pinray[d] = 0;
        if (r & checkers & sl) checkmask |= r;
        const uint64_t blk = r & our;
        if (blk) {
            const uint64_t r2 = ray_dir(d, kbb, empty | blk);
            if (r2 & sl & ~r) { pinned |= blk; pinray[d] = r2; }
        }
    }
    auto allowed = [&](int from) -> uint64_t {
        if (!((pinned >> from) & 1)) return ALL;
        uint64_t r = 0;
#pragma unroll
        for (int d = 0; d < 8; d++) r = ((pinray[d] >> from) & 1) && !r ? pinray[d] : r;
        return r;
    };
    const uint64_t sb = 1ULL << lane;
    if (tr && lane == 0) tr[8] = __builtin_amdgcn_s_memtime();
    *in_check = checkers != 0;
    const int nchk = popc64(checkers);
    // double check: only the king moves (and ep, whose attack test rejects it) -- empty target
    const uint64_t target = nchk == 0 ? ~our : (nchk == 1 ? checkmask : 0);
    const uint64_t ourP = p.bb[PAWN] & our;
    const uint64_t seventh = ourP & (us == 0 ? (0xFFULL << 48) : (0xFFULL << 8));
    const uint64_t single = (us == 0 ? (ourP << 8) : (ourP >> 8)) & empty;
    const uint64_t dbl = (us == 0 ? (single << 8) & (0xFFULL << 24) : (single >> 8) & (0xFFULL << 32)) & empty;
    const int home = us == 0 ? 0 : 56;
    // Generation groups in shakmaty order -- no check: ep, pawn captures, capture promotions,
    // pushes, push promotions, double pushes, N, B, R, Q, king, O-O, O-O-O; in check: ep, king,
    // then the non-king groups on the check mask.  Every lane is in at most one "main" group (the
    // piece on its square, or the pawn push landing on it) and computes its targets once; a move's
    // position is the count of all moves in earlier groups plus those of lower lanes in its own
    // group, from one ballot per group and one per bit of the count (no per-group passes).  The ep
    // captures (pawn lanes) come first, O-O / O-O-O (the king's lane) after the king moves.
    enum { G_CAP = 1, G_CPROMO, G_PUSH, G_PPROMO, G_DBL, G_N, G_B, G_R, G_Q, G_K, G_NONE };
    int grp = G_NONE, from = lane, flag = 0;
    uint64_t t = 0;
    const int role = piece_role_at(p, lane);
    if ((our >> lane) & 1) {
        const uint64_t allow = allowed(lane);
        if (role == PAWN) {
            grp = ((seventh >> lane) & 1) ? G_CPROMO : G_CAP;
            flag = grp == G_CPROMO ? PROMO_FLAG : 0;
            t = pawn_att(us, sb) & their & target & allow;
        } else if (role == KNIGHT) {
            grp = G_N;
            t = ((pinned >> lane) & 1) ? 0 : knight_att(sb) & target;
        } else if (role == KING) {
            grp = G_K;
            t = king_att(kbb) & ~our & ~attacked;
        } else {                                       // B, R, Q
            grp = G_B + (role - BISHOP);
            const uint64_t a = (role != ROOK ? bishop_att(sb, empty) : 0) | (role != BISHOP ? rook_att(sb, empty) : 0);
            t = a & target & allow;
        }
    } else if ((((single | dbl) & target) >> lane) & 1) {   // lane = a push's to-square
        const bool two = (dbl >> lane) & 1;
        from = us == 0 ? lane - (two ? 16 : 8) : lane + (two ? 16 : 8);
        grp = two ? G_DBL : (((BACKRANKS >> lane) & 1) ? G_PPROMO : G_PUSH);
        flag = grp == G_PPROMO ? PROMO_FLAG : 0;
        if ((allowed(from & 63) >> lane) & 1) t = sb;
    }
    // en passant (first in both orders), full attack test
    uint64_t ep_to = 0;
    if (p.ep < 64) {
        const uint64_t epbb = 1ULL << p.ep;
        const uint64_t capbb = 1ULL << (us == 0 ? p.ep - 8 : p.ep + 8);
        if (((ourP & pawn_att(them, epbb)) >> lane) & 1) {
            const uint64_t occ2 = (occ ^ sb ^ capbb) | epbb;
            const uint64_t att2 = (rook_att(kbb, ~occ2) & tR) | (bishop_att(kbb, ~occ2) & tB) |
                                  (knight_att(kbb) & tN) | (pawn_att(us, kbb) & tP & ~capbb);
            if (!att2) ep_to = epbb;
        }
    }
    const unsigned long long ep_mask = __ballot(ep_to != 0);
    *legal_ep = ep_mask != 0;
    const int n_ep = __popcll(ep_mask);
    // group order: rank of this lane's group; moves of all lanes whose group ranks lower come first
    const int cnt = t ? popc64(t) : 0;
    const int rank = nchk == 0 ? grp : (grp == G_K ? G_CAP : (grp < G_K ? grp + 1 : grp));
    unsigned long long before = 0, same = 0;         // lanes with a lower-ranked / the same group
#pragma unroll
    for (int g = G_CAP; g <= G_K; g++) {
        const int rg = nchk == 0 ? g : (g == G_K ? G_CAP : g + 1);
        const unsigned long long m = __ballot(grp == g && cnt > 0);
        before |= rg < rank ? m : 0ull;
        same = rg == rank ? m : same;
    }
    const unsigned long long below = same & ((1ull << lane) - 1ull);
    int mpos = n_ep, total = n_ep;
#pragma unroll
    for (int b = 0; b < 5; b++) {                     // counts <= 27: five bits
        const unsigned long long mb = __ballot((cnt >> b) & 1);
        mpos += (__popcll(mb & before) + __popcll(mb & below)) << b;
        total += __popcll(mb) << b;
    }
    if (tr && lane == 0) tr[9] = __builtin_amdgcn_s_memtime();
    // moves are staged in LDS as (from, to, flag) at their positions -- the serial per-lane loop
    // (up to 27 targets for a queen) is then a few instructions an iteration -- and written out as
    // edges by one lane per move (move index computed once per move, coalesced 16-byte stores)
    __shared__ uint32_t s_mv[NW][MAX_EDGES];
    uint32_t* mv = s_mv[(threadIdx.x >> 6) % NW];
    auto put = [&](int pos, int f, int to, int fl) { mv[pos] = (uint32_t)f | (uint32_t)to << 6 | (uint32_t)fl << 4; };
    if (ep_to) put(__popcll(ep_mask & ((1ull << lane) - 1ull)), lane, p.ep, 0);
    while (t) {                                        // this lane's main group, ascending to-squares
        put(mpos++, from, ctz64(t), flag);
        t &= t - 1;
    }
    // castling after the king moves (no check only): O-O then O-O-O, from the king's square
    if (nchk == 0) {
        const bool oo = (p.castling & (us == 0 ? 1 : 4)) && ksq == home + 4 && ((p.bb[ROOK] & our) >> (home + 7) & 1) &&
                        !(occ & (3ULL << (home + 5))) && !(attacked & (7ULL << (home + 4)));
        const bool ooo = (p.castling & (us == 0 ? 2 : 8)) && ksq == home + 4 && ((p.bb[ROOK] & our) >> home & 1) &&
                         !(occ & (7ULL << (home + 1))) && !(attacked & (7ULL << (home + 2)));
        if (lane == 0 && oo) put(total, ksq, home + 7, 0);
        if (lane == 0 && ooo) put(total + (oo ? 1 : 0), ksq, home, 0);
        total += (oo ? 1 : 0) + (ooo ? 1 : 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // this wave's LDS writes before its reads
    for (int o = lane; o < total; o += 64) {
        const uint32_t v = mv[o];
        Edge e;
        e.P = 0.0f; e.W = 0.0f; e.N = 0; e.child = CHILD_NONE;
        e.idx = (uint16_t)(move_index_bf((int)(v & 63u), (int)((v >> 6) & 63u), us) | (int)((v >> 4) & (uint32_t)PROMO_FLAG));
        out[o] = e;
    }
    return total;
}

// The rules part of an expansion, on the position the leaf's move led to (play_index, chess.rs:42):
// its legal moves as edges at `out` (gen_legal_wave), the legal-ep flag and repetition key, and
// outcome() (chess.rs:43-50).  Returns the outcome, *n = the edge count (distinct indices).  Shared
// with the rules probe (rules_probe.hip, az_rules_probe), which tests exactly this on the device.
template <int NW = GEN_WAVES>
__device__ __forceinline__ int leaf_rules(azc::Pos& c, Edge* __restrict__ out, int lane, int* n,
                                          unsigned long long* tr = nullptr, bool* in_check = nullptr) {
    bool chk = false, lep = false;
    *n = gen_legal_wave<NW>(c, out, lane, &chk, &lep, tr);
    c.flags = lep ? 1 : 0;
    c.rep_key = azc::rep_key_of(c);
    if (in_check) *in_check = chk;
    return azc::outcome(c, *n, chk);
}

template <int NW = GEN_WAVES>
__device__ __forceinline__ int expand_leaf_wave(const Engine& E, int g, int lane, int* nid_out, int step = -1) {
    // g is wave-uniform, and a provably uniform index would turn the per-game loads below into
    // scalar (s_load) reads; the leaf records were written by vector stores of another launch
    // (k_select), which the scalar cache does not see -- keep g in a VGPR so they stay vector loads
    g = vgpr_index(g);
    if (g >= E.G || !E.active[g] || E.leaf_kind[g] != LEAF_EVAL) return X_NONE;
    Node* nodes = game_nodes(E, g);
    Edge* edges = game_edges(E, g);
    azc::Pos* npos = game_npos(E, g);
    const int parent = E.leaf_node[g], eabs = E.leaf_edge[g];
    const int idx = edges[eabs].idx & azc::IDX_MASK;
    const azc::Pos pp = npos[parent];
    const int ebeg = E.edge_count[g];
    const int nid = E.node_count[g];
    const int pdepth = nodes[parent].depth;
    const int maxd = E.max_depth[g];
    const int hlen = E.hist_len[g];
    const int plen = E.leaf_len[g];
    const int* pn = E.path_node + (size_t)g * E.PMAX;
    unsigned long long* tr = nullptr;
#ifdef AZ_STEP_TRACE
    if (step == AZ_STEP_TRACE) tr = E.trace + (size_t)g * 16;
    if (tr && lane == 0) tr[10] = __builtin_amdgcn_s_memtime();
#endif
    azc::Pos c = azc::play_index(pp, idx);
#ifdef AZ_STEP_TRACE
    if (tr && lane == 0) tr[11] = __builtin_amdgcn_s_memtime();
#endif
    int n;
    int res = leaf_rules<NW>(c, edges + ebeg, lane, &n, tr);
#ifdef AZ_STEP_TRACE
    if (step == AZ_STEP_TRACE && lane == 0) E.trace[(size_t)g * 16 + 5] = __builtin_amdgcn_s_memtime();
#endif
    if (res == azc::ONGOING) {
        // earlier positions d plies back, d even, d <= halfmoves: d <= plen on the tree path
        // (pn[plen - d]), beyond it in the game history -- one candidate per lane
        const int hm = c.halfmoves;
        int cnt = 0;
        for (int d0 = 2; d0 <= hm; d0 += 128) {
            const int d = d0 + 2 * lane;
            bool eq = false;
            if (d <= hm) {
                if (d <= plen) eq = azc::chess_eq(npos[pn[plen - d]], c);
                else {
                    const int hi = hlen - 1 - d + plen;
                    if (hi >= 0) eq = azc::chess_eq(E.hist[(size_t)g * HMAX + hi], c);
                }
            }
            cnt += __popcll(__ballot(eq));
        }
        if (cnt + 1 >= azc::REPETITIONS || c.halfmoves >= azc::NUM_HALFMOVES || c.fullmoves >= azc::NUM_FULLMOVES)
            res = azc::DRAW;
    }
#ifdef AZ_STEP_TRACE
    if (step == AZ_STEP_TRACE && lane == 0) E.trace[(size_t)g * 16 + 6] = __builtin_amdgcn_s_memtime();
#endif
    if (res != azc::ONGOING) {
        if (lane == 0) {
            edges[eabs].child = res == azc::DRAW ? CHILD_DRAW : CHILD_WIN;
            E.leaf_kind[g] = res == azc::DRAW ? LEAF_DRAW : LEAF_WIN;
        }
        return X_TERMINAL;
    }
    if (nid >= E.NMAX || ebeg + n > E.EMAX) {
        if (lane == 0) {
            E.leaf_kind[g] = LEAF_DRAW;
            atomicAdd(&E.ctr->overflow, 1);
        }
        return X_NONE;
    }
    if (lane == 0) {
        Node nn;
        nn.edge_begin = (uint32_t)ebeg;
        nn.nedges = (uint16_t)n;
        nn.depth = (uint16_t)(pdepth + 1);
        nn.nsum = 0;
        nn.parent = parent;
        nodes[nid] = nn;
        npos[nid] = c;
        E.node_count[g] = nid + 1;
        E.edge_count[g] = ebeg + n;
        E.child_hdr[(size_t)g * E.EMAX + eabs] = (uint32_t)ebeg << 8 | (uint32_t)n;
        edges[eabs].child = nid;
        if (nn.depth > maxd) E.max_depth[g] = nn.depth;
    }
    if (E.cache_mask >= 0) {                                 // FEN cache lookup (tree.rs:214-219): probe = lane
        const uint64_t key = azc::fen_key(c);
        bool hit = false;
        int sl = 0;
        if (lane < CACHE_PROBES) {
            sl = (int)((key + (uint64_t)lane) & (uint64_t)E.cache_mask);
            hit = E.c_state[sl] == 2u && E.c_key[sl] == key && E.c_n[sl] == n && same_fen(E.c_pos[sl], c);
        }
        const unsigned long long hm = __ballot(hit);
        if (hm) {
            const int first = __builtin_ctzll(hm);
            sl = __shfl(sl, first, 64);
            const float* pri = E.c_pri + (size_t)sl * MAX_EDGES;
            for (int e = lane; e < n; e += 64) edges[ebeg + e].P = pri[e];
            if (lane == 0) {
                E.cached_value[g] = E.c_value[sl];
                E.leaf_kind[g] = LEAF_CACHED;
            }
            return X_CACHED;
        }
    }
    *nid_out = nid;
    return X_ROW;
}

// ------------------------------------------------------------------ backup
// the step's statistics (one thread of the grid): rows evaluated, then the row counter is
// cleared for step + 2
__device__ __forceinline__ void backup_stats(const Engine& E, int step) {
    int* rows = step_rows(E, step);
    const int n = load_fresh(rows);
    atomicAdd(&E.ctr->evals, (unsigned long long)n);
    if (step >= 0 && step < E.S) E.batch_hist[step] = n;
    *rows = 0;
}

// one wavefront backs up game g (active), one lane per tree level
__device__ __forceinline__ void backup_game(const Engine& E, int g, int lane) {
    Node* nodes = game_nodes(E, g);
    Edge* edges = game_edges(E, g);
    const int* pn = E.path_node + (size_t)g * E.PMAX;
    const int* pe = E.path_edge + (size_t)g * E.PMAX;
    // two rounds of dependent loads, not four: (1) the leaf record and the path's first 64 levels
    // (independent of the path length), (2) the leaf value and the edge / node records those levels
    // name (read speculatively at clamped indices: entries past the length are stale)
    const int lk = min(lane, E.PMAX - 1);
    const int p0e = min(max(pe[lk], 0), E.EMAX - 1), p0n = min(max(pn[lk], 0), E.NMAX - 1);
    const int kind = E.leaf_kind[g], len = E.leaf_len[g], row = E.leaf_row[g];
    const float ve = E.value[min(max(row, 0), E.G - 1)], vc = E.cached_value[g];
    Edge* ed0 = edges + p0e;
    Node* nd0 = nodes + p0n;
    const float w0 = ed0->W;
    const uint16_t n0 = ed0->N;
    const int s0 = nd0->nsum;
    // a second (never taken) use keeps the compiler from sinking the reads into the update below
    if (len == -1) E.trace[lane] = (unsigned long long)__builtin_bit_cast(unsigned, w0) + n0 + s0;
    const float v = kind == LEAF_EVAL ? ve : kind == LEAF_CACHED ? vc : (kind == LEAF_DRAW ? 0.0f : -1.0f);
    if (lane < len) {
        const float val = ((len - 1 - lane) & 1) ? v : -v;   // value = -child value per level
        ed0->W = w0 + val;
        ed0->N = (uint16_t)(n0 + 1);
        nd0->nsum = s0 + 1;
    }
    for (int k = lane + 64; k < len; k += 64) {
        const float val = ((len - 1 - k) & 1) ? v : -v;
        Edge* ed = edges + pe[k];
        ed->W = ed->W + val;
        ed->N = (uint16_t)(ed->N + 1);
        nodes[pn[k]].nsum += 1;
    }
    if (lane == 0) E.g_sims[g] += 1ull;                         // per-game slot, summed at readout
}

}  // namespace azi

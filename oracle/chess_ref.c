/*
 * chess_ref.c -- ORACLE (test infrastructure only, see az_oracle.h).
 *
 * Plain mailbox restatement of the reference's chess layer:
 *   chess.rs:13-27   GameState (position + pos_count multiset)
 *   chess.rs:36-63   play_move (is_legal -> play -> outcome -> repetition/50/200 rule)
 *   chess.rs:73-116  move_to_index
 *   chess.rs:118-171 index_to_move (UCI round trip, forced queen promotion)
 *   chess.rs:191-245 to_tensor (19 planes, side-to-move frame)
 * and of the shakmaty 0.29.0 semantics those call (legal_moves order, outcome(),
 * insufficient material, pseudo-legal / legal en-passant square, Chess equality).
 * Legality here is make-and-test (the product uses pin/check masks instead) and the
 * move list is sorted into shakmaty's generation order with an explicit key.
 */
#include "az_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { P = 1, N = 2, B = 3, R = 4, Q = 5, K = 6 };

static int sq_file(int s) { return s & 7; }
static int sq_rank(int s) { return s >> 3; }
static int on_board(int f, int r) { return f >= 0 && f < 8 && r >= 0 && r < 8; }
static int color_of(int pc) { return pc > 0 ? 0 : 1; }
static int role_of(int pc) { return pc > 0 ? pc : -pc; }
static int piece(int color, int role) { return color == 0 ? role : -role; }

void ref_startpos(ref_pos* p) {
    static const int back[8] = {R, N, B, Q, K, B, N, R};
    memset(p, 0, sizeof(*p));
    for (int f = 0; f < 8; f++) {
        p->sq[f] = (int8_t)back[f];
        p->sq[8 + f] = P;
        p->sq[48 + f] = -P;
        p->sq[56 + f] = (int8_t)-back[f];
    }
    p->turn = 0; p->castling = 15; p->ep = -1; p->halfmoves = 0; p->fullmoves = 1;
}

/* is square s attacked by pieces of color c (given the board) */
static int attacked_by(const int8_t* bd, int s, int c) {
    int f = sq_file(s), r = sq_rank(s);
    /* pawns: a pawn of color c on (f+-1, r -+ 1) */
    int pr = c == 0 ? r - 1 : r + 1;
    for (int df = -1; df <= 1; df += 2) {
        int ff = f + df;
        if (on_board(ff, pr) && bd[pr * 8 + ff] == piece(c, P)) return 1;
    }
    static const int kn[8][2] = {{1,2},{2,1},{2,-1},{1,-2},{-1,-2},{-2,-1},{-2,1},{-1,2}};
    for (int i = 0; i < 8; i++) {
        int ff = f + kn[i][0], rr = r + kn[i][1];
        if (on_board(ff, rr) && bd[rr * 8 + ff] == piece(c, N)) return 1;
    }
    for (int df = -1; df <= 1; df++) for (int dr = -1; dr <= 1; dr++) {
        if (!df && !dr) continue;
        int ff = f + df, rr = r + dr;
        if (on_board(ff, rr) && bd[rr * 8 + ff] == piece(c, K)) return 1;
    }
    static const int dirs[8][2] = {{0,1},{1,1},{1,0},{1,-1},{0,-1},{-1,-1},{-1,0},{-1,1}};
    for (int d = 0; d < 8; d++) {
        int diag = dirs[d][0] != 0 && dirs[d][1] != 0;
        int ff = f + dirs[d][0], rr = r + dirs[d][1];
        while (on_board(ff, rr)) {
            int pc = bd[rr * 8 + ff];
            if (pc) {
                if (color_of(pc) == c) {
                    int ro = role_of(pc);
                    if (ro == Q || (diag && ro == B) || (!diag && ro == R)) return 1;
                }
                break;
            }
            ff += dirs[d][0]; rr += dirs[d][1];
        }
    }
    return 0;
}

static int king_sq(const int8_t* bd, int c) {
    for (int s = 0; s < 64; s++) if (bd[s] == piece(c, K)) return s;
    return -1;
}

int ref_in_check(const ref_pos* p) {
    int k = king_sq(p->sq, p->turn);
    return k >= 0 && attacked_by(p->sq, k, 1 - p->turn);
}

/* shakmaty pseudo_legal_ep_square: the skipped square if a side-to-move pawn attacks it */
int ref_pseudo_legal_ep(const ref_pos* p) {
    if (p->ep < 0) return -1;
    int f = sq_file(p->ep), r = sq_rank(p->ep);
    int pr = p->turn == 0 ? r - 1 : r + 1;   /* our pawns sit one rank behind (our frame) */
    for (int df = -1; df <= 1; df += 2) {
        int ff = f + df;
        if (on_board(ff, pr) && p->sq[pr * 8 + ff] == piece(p->turn, P)) return p->ep;
    }
    return -1;
}

void ref_play_unchecked(ref_pos* p, ref_move m) {
    int us = p->turn;
    int pc = p->sq[m.from];
    int role = role_of(pc);
    int capture = 0;
    int new_ep = -1;
    if (m.kind == 2) {
        /* castle: king from e-file to g/c, rook from corner to f/d */
        int rank = us == 0 ? 0 : 7;
        int ks = m.to > m.from;
        p->sq[m.from] = 0; p->sq[m.to] = 0;
        p->sq[rank * 8 + (ks ? 6 : 2)] = (int8_t)piece(us, K);
        p->sq[rank * 8 + (ks ? 5 : 3)] = (int8_t)piece(us, R);
        p->castling &= us == 0 ? ~3 : ~12;
    } else if (m.kind == 1) {
        int cap = sq_rank(m.from) * 8 + sq_file(m.to);
        p->sq[cap] = 0;
        p->sq[m.to] = (int8_t)pc;
        p->sq[m.from] = 0;
        capture = 1;
    } else {
        capture = p->sq[m.to] != 0;
        p->sq[m.to] = (int8_t)(m.promo ? piece(us, m.promo) : pc);
        p->sq[m.from] = 0;
        if (role == P && (m.to - m.from == 16 || m.from - m.to == 16)) new_ep = (m.from + m.to) / 2;
        if (role == K) p->castling &= us == 0 ? ~3 : ~12;
        /* rook moved from / captured on a corner */
        if (m.from == 7 || m.to == 7) p->castling &= ~1;
        if (m.from == 0 || m.to == 0) p->castling &= ~2;
        if (m.from == 63 || m.to == 63) p->castling &= ~4;
        if (m.from == 56 || m.to == 56) p->castling &= ~8;
    }
    p->ep = new_ep;
    if (role == P || capture) p->halfmoves = 0; else p->halfmoves++;
    if (us == 1) p->fullmoves++;
    p->turn = 1 - us;
}

/* generation-order key (shakmaty position.rs legal_moves / gen_non_king / evasions) */
static int order_category(const ref_pos* p, ref_move m, int in_check) {
    int role = role_of(p->sq[m.from]);
    if (m.kind == 1) return 0;
    if (m.kind == 2) return m.to > m.from ? 11 : 12;
    int base = in_check ? 1 : 0;   /* in check: ep, king, then non-king */
    if (role == K) return in_check ? 1 : 10;
    int cat;
    if (role == P) {
        int capture = sq_file(m.from) != sq_file(m.to);
        int dbl = (m.to - m.from == 16) || (m.from - m.to == 16);
        if (capture) cat = m.promo ? 2 : 1;
        else if (dbl) cat = 5;
        else cat = m.promo ? 4 : 3;
    } else {
        cat = 6 + (role - N);   /* N 6, B 7, R 8, Q 9 */
    }
    return cat + base;
}

static int promo_rank(int promo) {
    switch (promo) { case Q: return 0; case R: return 1; case B: return 2; case N: return 3; default: return 0; }
}

typedef struct { int key; ref_move m; } keyed_move;
static int cmp_keyed(const void* a, const void* b) {
    return ((const keyed_move*)a)->key - ((const keyed_move*)b)->key;
}

static int pseudo_moves(const ref_pos* p, ref_move* out) {
    int n = 0, us = p->turn;
    const int8_t* bd = p->sq;
    int fwd = us == 0 ? 1 : -1;
    int start_rank = us == 0 ? 1 : 6, last_rank = us == 0 ? 7 : 0;
    static const int kn[8][2] = {{1,2},{2,1},{2,-1},{1,-2},{-1,-2},{-2,-1},{-2,1},{-1,2}};
    static const int dirs[8][2] = {{0,1},{1,1},{1,0},{1,-1},{0,-1},{-1,-1},{-1,0},{-1,1}};
    for (int s = 0; s < 64; s++) {
        int pc = bd[s];
        if (!pc || color_of(pc) != us) continue;
        int role = role_of(pc), f = sq_file(s), r = sq_rank(s);
        if (role == P) {
            int rr = r + fwd;
            if (!on_board(f, rr)) continue;
            if (!bd[rr * 8 + f]) {
                if (rr == last_rank) {
                    for (int pr = Q; pr >= N; pr--) out[n++] = (ref_move){(int16_t)s, (int16_t)(rr * 8 + f), (int8_t)pr, 0};
                } else {
                    out[n++] = (ref_move){(int16_t)s, (int16_t)(rr * 8 + f), 0, 0};
                    if (r == start_rank && !bd[(rr + fwd) * 8 + f])
                        out[n++] = (ref_move){(int16_t)s, (int16_t)((rr + fwd) * 8 + f), 0, 0};
                }
            }
            for (int df = -1; df <= 1; df += 2) {
                int ff = f + df;
                if (!on_board(ff, rr)) continue;
                int t = rr * 8 + ff;
                if (bd[t] && color_of(bd[t]) != us) {
                    if (rr == last_rank) {
                        for (int pr = Q; pr >= N; pr--) out[n++] = (ref_move){(int16_t)s, (int16_t)t, (int8_t)pr, 0};
                    } else out[n++] = (ref_move){(int16_t)s, (int16_t)t, 0, 0};
                } else if (t == p->ep && !bd[t]) {
                    out[n++] = (ref_move){(int16_t)s, (int16_t)t, 0, 1};
                }
            }
        } else if (role == N || role == K) {
            for (int i = 0; i < 8; i++) {
                int ff, rr;
                if (role == N) { ff = f + kn[i][0]; rr = r + kn[i][1]; }
                else { ff = f + dirs[i][0]; rr = r + dirs[i][1]; }
                if (!on_board(ff, rr)) continue;
                int t = rr * 8 + ff;
                if (bd[t] && color_of(bd[t]) == us) continue;
                out[n++] = (ref_move){(int16_t)s, (int16_t)t, 0, 0};
            }
        } else {
            for (int d = 0; d < 8; d++) {
                int diag = dirs[d][0] != 0 && dirs[d][1] != 0;
                if (role == B && !diag) continue;
                if (role == R && diag) continue;
                int ff = f + dirs[d][0], rr = r + dirs[d][1];
                while (on_board(ff, rr)) {
                    int t = rr * 8 + ff;
                    if (bd[t] && color_of(bd[t]) == us) break;
                    out[n++] = (ref_move){(int16_t)s, (int16_t)t, 0, 0};
                    if (bd[t]) break;
                    ff += dirs[d][0]; rr += dirs[d][1];
                }
            }
        }
    }
    /* castling (standard chess): king on e-file home square, rook on corner */
    int rank = us == 0 ? 0 : 7;
    int ksq = rank * 8 + 4;
    if (bd[ksq] == piece(us, K) && !attacked_by(bd, ksq, 1 - us)) {
        int kbit = us == 0 ? 1 : 4, qbit = us == 0 ? 2 : 8;
        if ((p->castling & kbit) && bd[rank * 8 + 7] == piece(us, R) && !bd[rank * 8 + 5] && !bd[rank * 8 + 6] &&
            !attacked_by(bd, rank * 8 + 5, 1 - us) && !attacked_by(bd, rank * 8 + 6, 1 - us))
            out[n++] = (ref_move){(int16_t)ksq, (int16_t)(rank * 8 + 7), 0, 2};
        if ((p->castling & qbit) && bd[rank * 8] == piece(us, R) && !bd[rank * 8 + 1] && !bd[rank * 8 + 2] &&
            !bd[rank * 8 + 3] && !attacked_by(bd, rank * 8 + 3, 1 - us) && !attacked_by(bd, rank * 8 + 2, 1 - us))
            out[n++] = (ref_move){(int16_t)ksq, (int16_t)(rank * 8), 0, 2};
    }
    return n;
}

int ref_legal_moves(const ref_pos* p, ref_move* out) {
    ref_move pm[REF_MAX_MOVES];
    keyed_move km[REF_MAX_MOVES];
    int np = pseudo_moves(p, pm), n = 0;
    int in_check = ref_in_check(p);
    for (int i = 0; i < np; i++) {
        ref_pos c = *p;
        ref_play_unchecked(&c, pm[i]);
        int k = king_sq(c.sq, p->turn);
        if (k >= 0 && attacked_by(c.sq, k, 1 - p->turn)) continue;
        int cat = order_category(p, pm[i], in_check);
        km[n].key = ((cat * 64 + pm[i].from) * 64 + pm[i].to) * 4 + promo_rank(pm[i].promo);
        km[n].m = pm[i];
        n++;
    }
    qsort(km, (size_t)n, sizeof(keyed_move), cmp_keyed);
    for (int i = 0; i < n; i++) out[i] = km[i].m;
    return n;
}

int ref_legal_ep(const ref_pos* p) {
    int ep = ref_pseudo_legal_ep(p);
    if (ep < 0) return -1;
    ref_move mv[REF_MAX_MOVES];
    int n = ref_legal_moves(p, mv);
    for (int i = 0; i < n; i++) if (mv[i].kind == 1) return ep;
    return -1;
}

/* shakmaty Board::has_insufficient_material(color), position = both colors */
static int insufficient_side(const ref_pos* p, int c) {
    int cnt[7] = {0}, tot = 0, other_nonkq = 0, pawns = 0, knights = 0, bishop_light = 0, bishop_dark = 0;
    for (int s = 0; s < 64; s++) {
        int pc = p->sq[s];
        if (!pc) continue;
        int ro = role_of(pc);
        if (ro == P) pawns++;
        if (ro == N) knights++;
        if (ro == B) { if (((sq_file(s) + sq_rank(s)) & 1) == 0) bishop_dark++; else bishop_light++; }
        if (color_of(pc) == c) { cnt[ro]++; tot++; }
        else if (ro != K && ro != Q) other_nonkq++;
    }
    if (cnt[P] || cnt[R] || cnt[Q]) return 0;
    if (cnt[N]) return tot <= 2 && other_nonkq == 0;
    if (cnt[B]) {
        int same_color = bishop_dark == 0 || bishop_light == 0;
        return same_color && pawns == 0 && knights == 0;
    }
    return 1;
}

int ref_insufficient_material(const ref_pos* p) {
    return insufficient_side(p, 0) && insufficient_side(p, 1);
}

/* shakmaty Position::outcome(): checkmate / stalemate / insufficient material */
int ref_outcome(const ref_pos* p) {
    ref_move mv[REF_MAX_MOVES];
    int n = ref_legal_moves(p, mv);
    if (n == 0) {
        if (ref_in_check(p)) return p->turn == 0 ? REF_BLACK_WINS : REF_WHITE_WINS;
        return REF_DRAW;
    }
    if (ref_insufficient_material(p)) return REF_DRAW;
    return REF_ONGOING;
}

uint64_t ref_perft(const ref_pos* p, int depth) {
    ref_move mv[REF_MAX_MOVES];
    int n = ref_legal_moves(p, mv);
    if (depth <= 1) return depth == 1 ? (uint64_t)n : 1;
    uint64_t t = 0;
    for (int i = 0; i < n; i++) {
        ref_pos c = *p;
        ref_play_unchecked(&c, mv[i]);
        t += ref_perft(&c, depth - 1);
    }
    return t;
}

/* ---- move index codec (chess.rs:73-171) ---- */
int ref_move_to_index(ref_move m, int turn) {
    int file = sq_file(m.from);
    int rank = turn == 1 ? 7 - sq_rank(m.from) : sq_rank(m.from);
    int dest_file = sq_file(m.to);
    int dest_rank = turn == 1 ? 7 - sq_rank(m.to) : sq_rank(m.to);
    int df = dest_file - file, dr = dest_rank - rank;
    int plane;
    if (df == 1 && dr == 2) plane = 0;
    else if (df == 2 && dr == 1) plane = 1;
    else if (df == 2 && dr == -1) plane = 2;
    else if (df == 1 && dr == -2) plane = 3;
    else if (df == -1 && dr == -2) plane = 4;
    else if (df == -2 && dr == -1) plane = 5;
    else if (df == -2 && dr == 1) plane = 6;
    else if (df == -1 && dr == 2) plane = 7;
    else if (df == 0 && dr >= 1) plane = 7 + dr;
    else if (df >= 1 && dr >= 1) plane = 14 + dr;
    else if (df >= 1 && dr == 0) plane = 21 + df;
    else if (df >= 1 && dr <= -1) plane = 28 + df;
    else if (df == 0 && dr <= -1) plane = 35 - dr;
    else if (df <= -1 && dr <= -1) plane = 42 - dr;
    else if (df <= -1 && dr == 0) plane = 49 - df;
    else if (df <= -1 && dr >= 1) plane = 56 - df;
    else { fprintf(stderr, "move_to_index: unreachable\n"); abort(); }
    return plane * 64 + rank * 8 + file;
}

static int same_move(ref_move a, ref_move b) {
    return a.from == b.from && a.to == b.to && a.promo == b.promo && a.kind == b.kind;
}

int ref_index_to_move(int index, const ref_pos* p, ref_move* out) {
    int plane = index / 64, sqi = index % 64;
    int from_file = sqi % 8, canon_rank = sqi / 8;
    int from_rank = p->turn == 1 ? 7 - canon_rank : canon_rank;
    int df, dr;
    static const int kn[8][2] = {{1,2},{2,1},{2,-1},{1,-2},{-1,-2},{-2,-1},{-2,1},{-1,2}};
    if (plane < 8) { df = kn[plane][0]; dr = kn[plane][1]; }
    else if (plane < 15) { df = 0; dr = plane - 7; }
    else if (plane < 22) { df = plane - 14; dr = plane - 14; }
    else if (plane < 29) { df = plane - 21; dr = 0; }
    else if (plane < 36) { df = plane - 28; dr = 28 - plane; }
    else if (plane < 43) { df = 0; dr = 35 - plane; }
    else if (plane < 50) { df = 42 - plane; dr = 42 - plane; }
    else if (plane < 57) { df = 49 - plane; dr = 0; }
    else { df = 56 - plane; dr = plane - 56; }
    if (p->turn == 1) dr = -dr;
    int dest_file = from_file + df, dest_rank = from_rank + dr;
    if (dest_file < 0 || dest_file > 7 || dest_rank < 0 || dest_rank > 7) return 0;
    int from = from_rank * 8 + from_file, to = dest_rank * 8 + dest_file;
    int pc = p->sq[from];
    if (!pc) return 0;                                   /* role_at(from)? */
    int role = role_of(pc);
    int promo = (role == P && (dest_rank == 0 || dest_rank == 7)) ? Q : 0;
    /* UciMove::to_move: king onto own castling rook -> Castle; e1g1-style -> Castle;
       pawn diagonal onto empty square -> EnPassant; else Normal.  Then is_legal. */
    ref_move cand = {(int16_t)from, (int16_t)to, (int8_t)promo, 0};
    int us = p->turn, home = us == 0 ? 0 : 7;
    if (role == K && color_of(pc) == us) {
        int kbit = us == 0 ? 1 : 4, qbit = us == 0 ? 2 : 8;
        if (((p->castling & kbit) && to == home * 8 + 7) || ((p->castling & qbit) && to == home * 8)) {
            if (p->sq[to] == piece(us, R)) cand.kind = 2;
        } else if (from == home * 8 + 4 && sq_rank(to) == home && (to - from == 2 || from - to == 2)) {
            cand.kind = 2;
            cand.to = (int16_t)(to > from ? home * 8 + 7 : home * 8);
        }
    } else if (role == P && sq_file(from) != sq_file(to) && !p->sq[to]) {
        cand.kind = 1;
    }
    ref_move mv[REF_MAX_MOVES];
    int n = ref_legal_moves(p, mv);
    for (int i = 0; i < n; i++) if (same_move(mv[i], cand)) { *out = cand; return 1; }
    return 0;
}

int ref_legal_indices(const ref_pos* p, int32_t* out) {
    ref_move mv[REF_MAX_MOVES];
    int n = ref_legal_moves(p, mv);
    for (int i = 0; i < n; i++) out[i] = ref_move_to_index(mv[i], p->turn);
    return n;
}

void ref_to_tensor(const ref_pos* p, float* t) {
    memset(t, 0, sizeof(float) * 19 * 64);
    int us = p->turn;
    for (int s = 0; s < 64; s++) {
        int pc = p->sq[s];
        if (!pc) continue;
        int off = color_of(pc) == us ? 0 : 6;
        int plane = role_of(pc) - 1 + off;
        int rank = us == 1 ? 7 - sq_rank(s) : sq_rank(s);
        t[plane * 64 + rank * 8 + sq_file(s)] = 1.0f;
    }
    int ck = us == 0 ? 1 : 4, cq = us == 0 ? 2 : 8, tk = us == 0 ? 4 : 1, tq = us == 0 ? 8 : 2;
    for (int i = 0; i < 64; i++) {
        if (p->castling & ck) t[12 * 64 + i] = 1.0f;
        if (p->castling & cq) t[13 * 64 + i] = 1.0f;
        if (p->castling & tk) t[14 * 64 + i] = 1.0f;
        if (p->castling & tq) t[15 * 64 + i] = 1.0f;
    }
    int ep = ref_pseudo_legal_ep(p);
    if (ep >= 0) {
        int rank = us == 1 ? 7 - sq_rank(ep) : sq_rank(ep);
        t[16 * 64 + rank * 8 + sq_file(ep)] = 1.0f;
    }
    float hm = (float)p->halfmoves / (float)REF_NUM_HALFMOVES;
    float fm = (float)p->fullmoves / (float)REF_NUM_FULLMOVES;
    for (int i = 0; i < 64; i++) { t[17 * 64 + i] = hm; t[18 * 64 + i] = fm; }
}

void ref_pos_bitboards(const ref_pos* p, uint64_t* bb) {
    memset(bb, 0, 8 * sizeof(uint64_t));
    for (int s = 0; s < 64; s++) {
        int pc = p->sq[s];
        if (!pc) continue;
        bb[role_of(pc) - 1] |= 1ULL << s;
        bb[6 + color_of(pc)] |= 1ULL << s;
    }
}

/* Key of FEN(pos, EnPassantMode::PseudoLegal): board, turn, castling, pseudo-legal ep, clocks.
 * Same definition as the product's az_fen_key (the cache / synthetic-evaluator key). */
uint64_t ref_fen_key(const ref_pos* p) {
    uint64_t bb[8];
    ref_pos_bitboards(p, bb);
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (int i = 0; i < 8; i++) h = ref_splitmix64(h ^ bb[i]);
    int ep = ref_pseudo_legal_ep(p);
    uint64_t meta = (uint64_t)p->turn | ((uint64_t)p->castling << 1) | ((uint64_t)(ep < 0 ? 64 : ep) << 5) |
                    ((uint64_t)p->halfmoves << 12) | ((uint64_t)p->fullmoves << 24);
    return ref_splitmix64(h ^ meta);
}

/* shakmaty Chess equality: board, turn, castling rights, legal ep square (counters ignored) */
int ref_chess_eq(const ref_pos* a, const ref_pos* b) {
    if (a->turn != b->turn || a->castling != b->castling) return 0;
    if (memcmp(a->sq, b->sq, 64) != 0) return 0;
    return ref_legal_ep(a) == ref_legal_ep(b);
}

/* ---- FEN ---- */
int ref_from_fen(const char* fen, ref_pos* p) {
    memset(p, 0, sizeof(*p));
    int r = 7, f = 0;
    const char* c = fen;
    for (; *c && *c != ' '; c++) {
        if (*c == '/') { r--; f = 0; continue; }
        if (*c >= '1' && *c <= '8') { f += *c - '0'; continue; }
        int role = 0;
        switch (*c | 32) { case 'p': role = P; break; case 'n': role = N; break; case 'b': role = B; break;
                           case 'r': role = R; break; case 'q': role = Q; break; case 'k': role = K; break; default: return -1; }
        if (r < 0 || f > 7) return -1;
        p->sq[r * 8 + f] = (int8_t)((*c >= 'a') ? -role : role);
        f++;
    }
    if (*c != ' ') return -1;
    c++;
    p->turn = (*c == 'b');
    c++;
    while (*c == ' ') c++;
    p->castling = 0;
    for (; *c && *c != ' '; c++) {
        if (*c == 'K') p->castling |= 1;
        if (*c == 'Q') p->castling |= 2;
        if (*c == 'k') p->castling |= 4;
        if (*c == 'q') p->castling |= 8;
    }
    /* drop rights whose king/rook are not on their home squares (shakmaty setup validation) */
    if (p->sq[4] != K) p->castling &= ~3;
    if (p->sq[7] != R) p->castling &= ~1;
    if (p->sq[0] != R) p->castling &= ~2;
    if (p->sq[60] != -K) p->castling &= ~12;
    if (p->sq[63] != -R) p->castling &= ~4;
    if (p->sq[56] != -R) p->castling &= ~8;
    while (*c == ' ') c++;
    p->ep = -1;
    if (*c && *c != '-') { p->ep = (c[1] - '1') * 8 + (c[0] - 'a'); c += 2; }
    else if (*c) c++;
    p->halfmoves = 0; p->fullmoves = 1;
    if (*c) sscanf(c, " %d %d", &p->halfmoves, &p->fullmoves);
    return 0;
}

int ref_to_fen(const ref_pos* p, char* out, int cap) {
    char buf[128];
    int n = 0;
    for (int r = 7; r >= 0; r--) {
        int empty = 0;
        for (int f = 0; f < 8; f++) {
            int pc = p->sq[r * 8 + f];
            if (!pc) { empty++; continue; }
            if (empty) { buf[n++] = (char)('0' + empty); empty = 0; }
            buf[n++] = "?PNBRQK"[role_of(pc)] | (pc < 0 ? 32 : 0);
        }
        if (empty) buf[n++] = (char)('0' + empty);
        if (r) buf[n++] = '/';
    }
    buf[n++] = ' '; buf[n++] = p->turn ? 'b' : 'w'; buf[n++] = ' ';
    if (!p->castling) buf[n++] = '-';
    if (p->castling & 1) buf[n++] = 'K';
    if (p->castling & 2) buf[n++] = 'Q';
    if (p->castling & 4) buf[n++] = 'k';
    if (p->castling & 8) buf[n++] = 'q';
    buf[n++] = ' ';
    int ep = ref_pseudo_legal_ep(p);
    if (ep < 0) buf[n++] = '-'; else { buf[n++] = (char)('a' + sq_file(ep)); buf[n++] = (char)('1' + sq_rank(ep)); }
    n += snprintf(buf + n, sizeof(buf) - (size_t)n, " %d %d", p->halfmoves, p->fullmoves);
    if (n + 1 > cap) return -1;
    memcpy(out, buf, (size_t)n + 1);
    return n;
}

/* ---- GameState (chess.rs:13-63) ---- */
static void game_reserve(ref_game* g, int need) {
    if (need <= g->cap) return;
    int cap = g->cap ? g->cap * 2 : 16;
    while (cap < need) cap *= 2;
    g->keys = (ref_pos*)realloc(g->keys, sizeof(ref_pos) * (size_t)cap);
    g->counts = (int32_t*)realloc(g->counts, sizeof(int32_t) * (size_t)cap);
    g->cap = cap;
}

void ref_game_new(ref_game* g) {
    memset(g, 0, sizeof(*g));
    ref_startpos(&g->position);
    game_reserve(g, 1);
    g->keys[0] = g->position;
    g->counts[0] = 1;
    g->n = 1;
}

/* a GameState whose repetition multiset starts at `start` (count 1), as GameState::new does
 * for the startpos (chess.rs:20-26); for searches from an arbitrary MCTree::new state (tree.rs:84) */
void ref_game_from(ref_game* g, const ref_pos* start) {
    ref_game_new(g);
    g->position = *start;
    g->keys[0] = *start;
}

/* Uniform random playouts from the startpos for rules parity tests (test data, not a reference
 * path): game k plays index_to_move(i) of a uniformly drawn legal index i (SplitMix64 of (seed,
 * k, ply)) through play_move (chess.rs:36-63) until the result is not Ongoing or max_plies.
 * Records every (parent position, index) pair; returns the count (<= cap). */
int64_t ref_random_playouts(uint64_t seed, int ngames, int max_plies, ref_pos* parents, int32_t* actions,
                            int64_t cap) {
    int64_t n = 0;
    for (int k = 0; k < ngames; k++) {
        ref_game g;
        ref_game_new(&g);
        for (int ply = 0; ply < max_plies; ply++) {
            int32_t idx[REF_MAX_MOVES];
            int nl = ref_legal_indices(&g.position, idx);
            if (nl == 0) break;
            uint64_t r = ref_splitmix64(ref_splitmix64(seed ^ ((uint64_t)k << 20)) ^ (uint64_t)ply);
            int a = idx[r % (uint64_t)nl];
            if (n < cap) { parents[n] = g.position; actions[n] = a; }
            n++;
            ref_move m;
            if (!ref_index_to_move(a, &g.position, &m)) break;
            if (ref_play_move(&g, m) != REF_ONGOING) break;
        }
        ref_game_free(&g);
    }
    return n;
}

/* Packed view of positions for tests: bitboards P N B R Q K white black, and meta = {turn, castling,
 * pseudo-legal ep (64 = none), halfmoves, fullmoves} -- the fields of the product's az_pos. */
void ref_pack(const ref_pos* p, int64_t n, uint64_t* bb, int32_t* meta) {
    for (int64_t i = 0; i < n; i++) {
        ref_pos_bitboards(&p[i], bb + 8 * i);
        int ep = ref_pseudo_legal_ep(&p[i]);
        int32_t* m = meta + 5 * i;
        m[0] = p[i].turn; m[1] = p[i].castling; m[2] = ep < 0 ? 64 : ep;
        m[3] = p[i].halfmoves; m[4] = p[i].fullmoves;
    }
}

/* The rules answers for n items (test data): child = parent with index_to_move(action) played
 * (action < 0: the parent itself), its legal indices with duplicates (tree.rs:86-89), outcome(),
 * in-check, legal ep square (-1 = none), FEN key and to_tensor planes.  Returns the number of
 * items whose action was not legal (their outputs are the parent's). */
int64_t ref_rules_batch(const ref_pos* parent, const int32_t* action, int64_t n, ref_pos* child, int32_t* moves,
                        int32_t* nmoves, int32_t* outcome, int32_t* in_check, int32_t* legal_ep, uint64_t* fen_key,
                        float* planes) {
    int64_t bad = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+:bad)
    for (int64_t i = 0; i < n; i++) {
        ref_pos c = parent[i];
        if (action[i] >= 0) {
            ref_move m;
            if (ref_index_to_move(action[i], &c, &m)) ref_play_unchecked(&c, m);
            else bad++;
        }
        child[i] = c;
        nmoves[i] = ref_legal_indices(&c, moves + (size_t)i * REF_MAX_MOVES);
        outcome[i] = ref_outcome(&c);
        in_check[i] = ref_in_check(&c);
        legal_ep[i] = ref_legal_ep(&c);
        fen_key[i] = ref_fen_key(&c);
        ref_to_tensor(&c, planes + (size_t)i * 19 * 64);
    }
    return bad;
}

void ref_game_clone(ref_game* dst, const ref_game* src) {
    memset(dst, 0, sizeof(*dst));
    dst->position = src->position;
    game_reserve(dst, src->n > 0 ? src->n : 1);
    memcpy(dst->keys, src->keys, sizeof(ref_pos) * (size_t)src->n);
    memcpy(dst->counts, src->counts, sizeof(int32_t) * (size_t)src->n);
    dst->n = src->n;
}

void ref_game_free(ref_game* g) {
    free(g->keys); free(g->counts);
    memset(g, 0, sizeof(*g));
}

int ref_play_move(ref_game* g, ref_move m) {
    ref_move mv[REF_MAX_MOVES];
    int n = ref_legal_moves(&g->position, mv), legal = 0;
    for (int i = 0; i < n; i++) if (same_move(mv[i], m)) { legal = 1; break; }
    if (!legal) return REF_ILLEGAL;                                  /* chess.rs:38-39 */
    ref_play_unchecked(&g->position, m);                            /* chess.rs:42 */
    int oc = ref_outcome(&g->position);                             /* chess.rs:43-50 */
    if (oc != REF_ONGOING) return oc;
    int idx = -1;                                                    /* chess.rs:52-53 */
    for (int i = 0; i < g->n; i++) if (ref_chess_eq(&g->keys[i], &g->position)) { idx = i; break; }
    if (idx < 0) {
        game_reserve(g, g->n + 1);
        g->keys[g->n] = g->position;
        g->counts[g->n] = 0;
        idx = g->n++;
    }
    int count = ++g->counts[idx];
    if (count < REF_REPETITIONS && g->position.halfmoves < REF_NUM_HALFMOVES &&
        g->position.fullmoves < REF_NUM_FULLMOVES)                   /* chess.rs:55-60 */
        return REF_ONGOING;
    return REF_DRAW;
}

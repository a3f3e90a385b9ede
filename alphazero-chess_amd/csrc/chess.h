// chess.h -- bitboard chess core of the engine, compiled for gfx950 device code and
// for the host side of libaz (az_pos_* / az_game_* entry points).
//
// Replaces the reference's chess layer and the shakmaty 0.29 calls it makes:
//   chess.rs:36-63   play_move: legality -> play -> outcome() -> repetition / 50-move /
//                    200-fullmove draw
//   chess.rs:73-116  move_to_index        chess.rs:118-171 index_to_move
//   chess.rs:191-245 to_tensor (19 planes, side-to-move frame)
//   shakmaty legal_moves() generation order (ep, pawns, N, B, R, Q, king, O-O, O-O-O;
//   in check: ep, king, then blocks/captures), outcome(), insufficient material,
//   pseudo-legal / legal ep square, Chess equality (board, turn, castling, legal ep).
// Branch-light GPU formulation: Kogge-Stone occluded fills for sliders (no tables),
// set-wise attack maps, pin rays from the king -- one lane runs one position.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define AZ_HD __host__ __device__ __forceinline__
#else
#define AZ_HD static inline
#endif

namespace azc {

enum Role { PAWN = 0, KNIGHT = 1, BISHOP = 2, ROOK = 3, QUEEN = 4, KING = 5 };
enum { WHITE_BB = 6, BLACK_BB = 7 };
enum { ONGOING = 0, DRAW = 1, WHITE_WINS = 2, BLACK_WINS = 3, ILLEGAL = -1 };
enum { NUM_HALFMOVES = 100, NUM_FULLMOVES = 200, REPETITIONS = 3 };   // chess.rs:9-11
enum { PROMO_FLAG = 0x1000, IDX_MASK = 0x0FFF };

struct Pos {                       // == az_pos (include/az.h), 80 bytes
    uint64_t bb[8];
    uint8_t turn, castling, ep, flags;
    uint16_t halfmoves, fullmoves;
    uint64_t rep_key;
};

AZ_HD uint64_t side_bb(const Pos& p, int color) { return color ? p.bb[BLACK_BB] : p.bb[WHITE_BB]; }
AZ_HD uint64_t role_bb(const Pos& p, int role) {
    uint64_t r = p.bb[0];
#pragma unroll
    for (int i = 1; i < 6; i++) r = role == i ? p.bb[i] : r;
    return r;
}

constexpr uint64_t FILE_A = 0x0101010101010101ULL;
constexpr uint64_t FILE_H = FILE_A << 7;
constexpr uint64_t NOT_A = ~FILE_A;
constexpr uint64_t NOT_H = ~FILE_H;
constexpr uint64_t NOT_AB = ~(FILE_A | (FILE_A << 1));
constexpr uint64_t NOT_GH = ~(FILE_H | (FILE_H >> 1));
constexpr uint64_t RANK_1 = 0xFFULL;
constexpr uint64_t RANK_8 = 0xFFULL << 56;
constexpr uint64_t BACKRANKS = RANK_1 | RANK_8;
constexpr uint64_t DARK = 0xAA55AA55AA55AA55ULL;
constexpr uint64_t ALL = ~0ULL;

AZ_HD int ctz64(uint64_t b) { return __builtin_ctzll(b); }
AZ_HD int clz64(uint64_t b) { return __builtin_clzll(b); }
AZ_HD int popc64(uint64_t b) { return __builtin_popcountll(b); }
// bitboard accessors with a run-time colour / role: selects over static indices, so a Pos in
// registers is never indexed dynamically (which would move it to scratch memory on the GPU)
struct Pos;
AZ_HD uint64_t side_bb(const Pos& p, int color);
AZ_HD uint64_t role_bb(const Pos& p, int role);

AZ_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

template <int S> AZ_HD uint64_t shl(uint64_t b) { return S > 0 ? (b << (S > 0 ? S : 0)) : (b >> (S < 0 ? -S : 0)); }

// Kogge-Stone occluded fill in one direction (S = shift, M = wrap mask)
template <int S, uint64_t M> AZ_HD uint64_t occl(uint64_t gen, uint64_t pro) {
    pro &= M;
    gen |= pro & shl<S>(gen);
    pro &= shl<S>(pro);
    gen |= pro & shl<2 * S>(gen);
    pro &= shl<2 * S>(pro);
    gen |= pro & shl<4 * S>(gen);
    return gen;
}
template <int S, uint64_t M> AZ_HD uint64_t ray(uint64_t sliders, uint64_t empty) {
    return shl<S>(occl<S, M>(sliders, empty)) & M;
}
// direction d: 0 N, 1 NE, 2 E, 3 SE, 4 S, 5 SW, 6 W, 7 NW
AZ_HD uint64_t ray_dir(int d, uint64_t s, uint64_t empty) {
    switch (d) {
        case 0: return ray<8, ALL>(s, empty);
        case 1: return ray<9, NOT_A>(s, empty);
        case 2: return ray<1, NOT_A>(s, empty);
        case 3: return ray<-7, NOT_A>(s, empty);
        case 4: return ray<-8, ALL>(s, empty);
        case 5: return ray<-9, NOT_H>(s, empty);
        case 6: return ray<-1, NOT_H>(s, empty);
        default: return ray<7, NOT_H>(s, empty);
    }
}
AZ_HD uint64_t rook_att(uint64_t s, uint64_t empty) {
    return ray<8, ALL>(s, empty) | ray<-8, ALL>(s, empty) | ray<1, NOT_A>(s, empty) | ray<-1, NOT_H>(s, empty);
}
AZ_HD uint64_t bishop_att(uint64_t s, uint64_t empty) {
    return ray<9, NOT_A>(s, empty) | ray<7, NOT_H>(s, empty) | ray<-7, NOT_A>(s, empty) | ray<-9, NOT_H>(s, empty);
}
AZ_HD uint64_t knight_att(uint64_t b) {
    uint64_t l1 = (b >> 1) & NOT_H, l2 = (b >> 2) & NOT_GH;
    uint64_t r1 = (b << 1) & NOT_A, r2 = (b << 2) & NOT_AB;
    uint64_t h1 = l1 | r1, h2 = l2 | r2;
    return (h1 << 16) | (h1 >> 16) | (h2 << 8) | (h2 >> 8);
}
AZ_HD uint64_t king_att(uint64_t b) {
    uint64_t att = ((b << 1) & NOT_A) | ((b >> 1) & NOT_H);
    b |= att;
    return att | (b << 8) | (b >> 8);
}
AZ_HD uint64_t pawn_att(int color, uint64_t b) {
    return color == 0 ? (((b << 9) & NOT_A) | ((b << 7) & NOT_H)) : (((b >> 7) & NOT_A) | ((b >> 9) & NOT_H));
}

AZ_HD int piece_role_at(const Pos& p, int sq) {
    const uint64_t m = 1ULL << sq;
    int role = -1;
#pragma unroll
    for (int r = 5; r >= 0; r--) role = (p.bb[r] & m) ? r : role;
    return role;
}

// chess.rs:73-116 move_to_index (to = rook square for castling, shakmaty Move::to())
AZ_HD int move_index(int from, int to, int turn) {
    int file = from & 7, rank = turn ? 7 - (from >> 3) : (from >> 3);
    int dfile = to & 7, drank = turn ? 7 - (to >> 3) : (to >> 3);
    int df = dfile - file, dr = drank - rank;
    int plane;
    if (df == 1 && dr == 2) plane = 0;
    else if (df == 2 && dr == 1) plane = 1;
    else if (df == 2 && dr == -1) plane = 2;
    else if (df == 1 && dr == -2) plane = 3;
    else if (df == -1 && dr == -2) plane = 4;
    else if (df == -2 && dr == -1) plane = 5;
    else if (df == -2 && dr == 1) plane = 6;
    else if (df == -1 && dr == 2) plane = 7;
    else if (df == 0) plane = dr > 0 ? 7 + dr : 35 - dr;
    else if (dr == 0) plane = df > 0 ? 21 + df : 49 - df;
    else if (df > 0) plane = dr > 0 ? 14 + dr : 28 + df;
    else plane = dr < 0 ? 42 - dr : 56 - df;
    return plane * 64 + rank * 8 + file;
}

// plane -> (df, dr) in the mover's frame (chess.rs:131-150)
AZ_HD void plane_delta(int plane, int& df, int& dr) {
    if (plane < 8) {                 // (1,2) (2,1) (2,-1) (1,-2) (-1,-2) (-2,-1) (-2,1) (-1,2), as selects
        const int a = (plane == 0 || plane == 3 || plane == 4 || plane == 7) ? 1 : 2;
        df = plane < 4 ? a : -a;
        dr = (plane == 0 || plane == 7) ? 2 : (plane == 1 || plane == 6) ? 1 : (plane == 2 || plane == 5) ? -1 : -2;
    } else if (plane < 15) { df = 0; dr = plane - 7; }
    else if (plane < 22) { df = plane - 14; dr = plane - 14; }
    else if (plane < 29) { df = plane - 21; dr = 0; }
    else if (plane < 36) { df = plane - 28; dr = 28 - plane; }
    else if (plane < 43) { df = 0; dr = 35 - plane; }
    else if (plane < 50) { df = 42 - plane; dr = 42 - plane; }
    else if (plane < 57) { df = 49 - plane; dr = 0; }
    else { df = 56 - plane; dr = plane - 56; }
}

AZ_HD bool insufficient_side(const Pos& p, int c) {
    uint64_t ours = side_bb(p, c), theirs = side_bb(p, c ^ 1);
    if (ours & (p.bb[PAWN] | p.bb[ROOK] | p.bb[QUEEN])) return false;
    if (ours & p.bb[KNIGHT]) return popc64(ours) <= 2 && (theirs & ~p.bb[KING] & ~p.bb[QUEEN]) == 0;
    if (ours & p.bb[BISHOP]) {
        bool same = (p.bb[BISHOP] & DARK) == 0 || (p.bb[BISHOP] & ~DARK) == 0;
        return same && p.bb[PAWN] == 0 && p.bb[KNIGHT] == 0;
    }
    return true;
}
AZ_HD bool insufficient_material(const Pos& p) { return insufficient_side(p, 0) && insufficient_side(p, 1); }

// pseudo-legal ep: a side-to-move pawn attacks the skipped square (shakmaty)
AZ_HD uint8_t pseudo_ep(const Pos& p, int ep_sq) {
    if (ep_sq >= 64) return 64;
    uint64_t ours = p.bb[PAWN] & side_bb(p, p.turn);
    return (pawn_att(p.turn ^ 1, 1ULL << ep_sq) & ours) ? (uint8_t)ep_sq : (uint8_t)64;
}

AZ_HD uint64_t fen_key(const Pos& p) {      // key of FEN(pos, PseudoLegal) (tree.rs:214)
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (int i = 0; i < 8; i++) h = splitmix64(h ^ p.bb[i]);
    uint64_t meta = (uint64_t)p.turn | ((uint64_t)p.castling << 1) | ((uint64_t)p.ep << 5) |
                    ((uint64_t)p.halfmoves << 12) | ((uint64_t)p.fullmoves << 24);
    return splitmix64(h ^ meta);
}
AZ_HD uint64_t rep_key_of(const Pos& p) {   // key of shakmaty Chess equality
    uint64_t h = 0x13198A2E03707344ULL;
    for (int i = 0; i < 8; i++) h = splitmix64(h ^ p.bb[i]);
    uint64_t lep = (p.flags & 1) ? p.ep : 64;
    return splitmix64(h ^ ((uint64_t)p.turn | ((uint64_t)p.castling << 1) | (lep << 5)));
}
AZ_HD bool chess_eq(const Pos& a, const Pos& b) {
    if (a.rep_key != b.rep_key || a.turn != b.turn || a.castling != b.castling) return false;
    for (int i = 0; i < 8; i++) if (a.bb[i] != b.bb[i]) return false;
    uint8_t la = (a.flags & 1) ? a.ep : 64, lb = (b.flags & 1) ? b.ep : 64;
    return la == lb;
}

// Legal move generation in shakmaty 0.29 legal_moves() order.  Calls sink(idx) once per
// distinct move index: under-promotions share the queen promotion's index and are
// reported once with PROMO_FLAG (4 entries in the reference's `moves`, tree.rs:86-89).
// Returns the number of distinct indices; *in_check, *legal_ep set.
template <class Sink> AZ_HD int gen_legal(const Pos& p, Sink& sink, bool* in_check, bool* legal_ep) {
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
    // pins and check rays from the king
    uint64_t pinned = 0, pinray[8], checkmask = checkers;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        uint64_t r = ray_dir(d, kbb, empty);
        const uint64_t sl = (d & 1) ? tB : tR;
        pinray[d] = 0;
        if (r & checkers & sl) checkmask |= r;
        uint64_t blk = r & our;
        if (blk) {
            uint64_t r2 = ray_dir(d, kbb, empty | blk);
            if (r2 & sl & ~r) { pinned |= blk; pinray[d] = r2; }
        }
    }
    int n = 0;
    *in_check = checkers != 0;
    *legal_ep = false;
    // en passant first (gen_en_passant), legality by a full attack test
    if (p.ep < 64) {
        const uint64_t epbb = 1ULL << p.ep;
        const int capsq = us == 0 ? p.ep - 8 : p.ep + 8;
        const uint64_t capbb = 1ULL << capsq;
        uint64_t fr = p.bb[PAWN] & our & pawn_att(them, epbb);
        while (fr) {
            const int from = ctz64(fr);
            fr &= fr - 1;
            const uint64_t occ2 = (occ ^ (1ULL << from) ^ capbb) | epbb;
            const uint64_t att2 = (rook_att(kbb, ~occ2) & tR) | (bishop_att(kbb, ~occ2) & tB) |
                                  (knight_att(kbb) & tN) | (pawn_att(us, kbb) & tP & ~capbb);
            if (!att2) { sink(move_index(from, p.ep, us)); n++; *legal_ep = true; }
        }
    }
    const int nchk = popc64(checkers);
    auto king_moves = [&]() {
        uint64_t t = king_att(kbb) & ~our & ~attacked;
        while (t) { const int to = ctz64(t); t &= t - 1; sink(move_index(ksq, to, us)); n++; }
    };
    auto allowed = [&](int from) -> uint64_t {
        if (!((pinned >> from) & 1)) return ALL;
        uint64_t r = 0;                                // pinray[] stays in registers (no early exit)
#pragma unroll
        for (int d = 0; d < 8; d++) r = ((pinray[d] >> from) & 1) && !r ? pinray[d] : r;
        return r;
    };
    auto non_king = [&](uint64_t target) {
        const uint64_t ourP = p.bb[PAWN] & our;
        const uint64_t seventh = ourP & (us == 0 ? (0xFFULL << 48) : (0xFFULL << 8));
        uint64_t fr = ourP & ~seventh;
        while (fr) {                                   // captures
            const int from = ctz64(fr); fr &= fr - 1;
            uint64_t t = pawn_att(us, 1ULL << from) & their & target & allowed(from);
            while (t) { const int to = ctz64(t); t &= t - 1; sink(move_index(from, to, us)); n++; }
        }
        fr = seventh;
        while (fr) {                                   // capture promotions
            const int from = ctz64(fr); fr &= fr - 1;
            uint64_t t = pawn_att(us, 1ULL << from) & their & target & allowed(from);
            while (t) { const int to = ctz64(t); t &= t - 1; sink(move_index(from, to, us) | PROMO_FLAG); n++; }
        }
        const uint64_t single = (us == 0 ? (ourP << 8) : (ourP >> 8)) & empty;
        const uint64_t dbl = (us == 0 ? (single << 8) & (0xFFULL << 24) : (single >> 8) & (0xFFULL << 32)) & empty;
        uint64_t t = single & target & ~BACKRANKS;
        while (t) {
            const int to = ctz64(t); t &= t - 1;
            const int from = us == 0 ? to - 8 : to + 8;
            if ((allowed(from) >> to) & 1) { sink(move_index(from, to, us)); n++; }
        }
        t = single & target & BACKRANKS;
        while (t) {
            const int to = ctz64(t); t &= t - 1;
            const int from = us == 0 ? to - 8 : to + 8;
            if ((allowed(from) >> to) & 1) { sink(move_index(from, to, us) | PROMO_FLAG); n++; }
        }
        t = dbl & target;
        while (t) {
            const int to = ctz64(t); t &= t - 1;
            const int from = us == 0 ? to - 16 : to + 16;
            if ((allowed(from) >> to) & 1) { sink(move_index(from, to, us)); n++; }
        }
        fr = p.bb[KNIGHT] & our & ~pinned;
        while (fr) {
            const int from = ctz64(fr); fr &= fr - 1;
            uint64_t tt = knight_att(1ULL << from) & target;
            while (tt) { const int to = ctz64(tt); tt &= tt - 1; sink(move_index(from, to, us)); n++; }
        }
#pragma unroll
        for (int role = BISHOP; role <= QUEEN; role++) {
            fr = role_bb(p, role) & our;
            while (fr) {
                const int from = ctz64(fr); fr &= fr - 1;
                const uint64_t sb = 1ULL << from;
                uint64_t a = role == BISHOP ? bishop_att(sb, empty)
                           : role == ROOK ? rook_att(sb, empty) : (bishop_att(sb, empty) | rook_att(sb, empty));
                uint64_t tt = a & target & allowed(from);
                while (tt) { const int to = ctz64(tt); tt &= tt - 1; sink(move_index(from, to, us)); n++; }
            }
        }
    };
    if (nchk == 0) {
        non_king(~our);
        king_moves();
        const int home = us == 0 ? 0 : 56;
        const uint8_t kbit = us == 0 ? 1 : 4, qbit = us == 0 ? 2 : 8;
        if ((p.castling & kbit) && ksq == home + 4 && ((p.bb[ROOK] & our) >> (home + 7) & 1) &&
            !(occ & (3ULL << (home + 5))) && !(attacked & (7ULL << (home + 4)))) {
            sink(move_index(ksq, home + 7, us)); n++;
        }
        if ((p.castling & qbit) && ksq == home + 4 && ((p.bb[ROOK] & our) >> home & 1) &&
            !(occ & (7ULL << (home + 1))) && !(attacked & (7ULL << (home + 2)))) {
            sink(move_index(ksq, home, us)); n++;
        }
    } else {
        king_moves();
        if (nchk == 1) non_king(checkmask);
    }
    return n;
}

struct NullSink { AZ_HD void operator()(int) {} };

// index_to_move (chess.rs:118-171, UciMove::to_move) + play_unchecked for an index known
// to be legal. Under-promotion indices play the queen promotion (chess.rs:165-167).
AZ_HD Pos play_index(const Pos& p, int idx) {
    const int us = p.turn, them = us ^ 1;
    const int plane = idx >> 6, s = idx & 63;
    const int file = s & 7, crank = s >> 3;
    const int frank = us ? 7 - crank : crank;
    int df, dr;
    plane_delta(plane, df, dr);
    if (us) dr = -dr;
    const int from = frank * 8 + file, to = (frank + dr) * 8 + file + df;
    Pos c = p;
    const uint64_t fb = 1ULL << from, tb = 1ULL << to;
    const int role = piece_role_at(p, from);
    const uint64_t our = side_bb(p, us);
    const int home = us == 0 ? 0 : 56;
    bool is_castle = false;
    if (role == KING) {
        const uint8_t kbit = us == 0 ? 1 : 4, qbit = us == 0 ? 2 : 8;
        if ((our & p.bb[ROOK] & tb) && (((p.castling & kbit) && to == home + 7) || ((p.castling & qbit) && to == home)))
            is_castle = true;
    }
    bool capture = false;
    int new_ep = 64;
    // colour / role updates as masks applied to every bitboard (static indices only)
    uint64_t xor_us = 0, clr_them = 0, clr_all = 0;
    uint64_t role_clr[6] = {0, 0, 0, 0, 0, 0}, role_set[6] = {0, 0, 0, 0, 0, 0};
    if (is_castle) {
        const bool ks = to > from;
        const int kto = home + (ks ? 6 : 2), rto = home + (ks ? 5 : 3);
        c.bb[KING] ^= fb | (1ULL << kto);
        c.bb[ROOK] ^= tb | (1ULL << rto);
        xor_us = fb | tb | (1ULL << kto) | (1ULL << rto);
        c.castling &= us == 0 ? ~3 : ~12;
    } else {
        if (side_bb(p, them) & tb) {                  // capture
            capture = true;
            clr_all = tb;
            clr_them = tb;
        } else if (role == PAWN && df != 0) {          // en passant
            capture = true;
            const uint64_t cb = 1ULL << (us == 0 ? to - 8 : to + 8);
            role_clr[PAWN] = cb;
            clr_them = cb;
        }
        const bool promo = role == PAWN && (tb & BACKRANKS);
        const int placed = promo ? QUEEN : role;
#pragma unroll
        for (int r = 0; r < 6; r++) {
            if (r == role) role_clr[r] |= fb;
            if (r == placed) role_set[r] |= tb;
        }
        xor_us = fb | tb;
        if (role == KING) c.castling &= us == 0 ? ~3 : ~12;
        if (from == 7 || to == 7) c.castling &= ~1;
        if (from == 0 || to == 0) c.castling &= ~2;
        if (from == 63 || to == 63) c.castling &= ~4;
        if (from == 56 || to == 56) c.castling &= ~8;
        if (role == PAWN && (dr == 2 || dr == -2)) new_ep = (from + to) >> 1;
    }
#pragma unroll
    for (int r = 0; r < 6; r++) c.bb[r] = ((c.bb[r] & ~clr_all) & ~role_clr[r]) | role_set[r];
    c.bb[WHITE_BB] = (c.bb[WHITE_BB] ^ (us == 0 ? xor_us : 0)) & ~(us == 0 ? 0 : clr_them);
    c.bb[BLACK_BB] = (c.bb[BLACK_BB] ^ (us == 1 ? xor_us : 0)) & ~(us == 1 ? 0 : clr_them);
    c.turn = (uint8_t)them;
    c.halfmoves = (role == PAWN || capture) ? 0 : (uint16_t)(p.halfmoves + 1);
    if (us == 1) c.fullmoves = (uint16_t)(p.fullmoves + 1);
    c.ep = pseudo_ep(c, new_ep);
    c.flags = 0;
    c.rep_key = 0;
    return c;
}

// Fill flags (legal ep) and rep_key of a freshly made position; returns legal move count.
AZ_HD int finalize(Pos& p, bool* in_check) {
    NullSink ns;
    bool lep = false;
    int n = gen_legal(p, ns, in_check, &lep);
    p.flags = lep ? 1 : 0;
    p.rep_key = rep_key_of(p);
    return n;
}

// a, b and c on one rank, file, diagonal or anti-diagonal (shakmaty attacks::aligned: c on the
// line through a and b)
AZ_HD bool aligned3(int a, int b, int c) {
    auto r = [](int x) { return x >> 3; };
    auto f = [](int x) { return x & 7; };
    return (r(a) == r(b) && r(b) == r(c)) || (f(a) == f(b) && f(b) == f(c)) ||
           (r(a) - f(a) == r(b) - f(b) && r(b) - f(b) == r(c) - f(c)) ||
           (r(a) + f(a) == r(b) + f(b) && r(b) + f(b) == r(c) + f(c));
}

// Why a caller's position is not one shakmaty's Chess::from_setup accepts (its PositionErrorKinds:
// bitboard consistency, one king per side, too much material, pawns on a back rank, invalid
// castling rights / ep square, the side not to move in check, impossible check), or nullptr.
// The reference only ever reaches positions by legal play from Chess::default() (training.rs:344),
// so these are exactly the positions it can hold; the engine sizes a node's edges for 218 legal
// moves (az_internal.h MAX_EDGES, search.hip EMAX), which every accepted position respects.
// raw_ep: a FEN's ep square as written (shakmaty validates that one, EnPassant::from_setup; the
// pseudo-legal square p.ep derives from it is what the position keeps); -1: p.ep itself, which must
// then also be pseudo-legal (the az_pos invariant for positions passed in as records).
// Restated from shakmaty 0.29's published validate(); parity unpinned (no fixture holds it).
inline const char* setup_error(const Pos& p, int raw_ep = -1) {
    const uint64_t w = p.bb[WHITE_BB], b = p.bb[BLACK_BB];
    if (w & b) return "white and black bitboards overlap";
    uint64_t roles = 0;
    for (int r = 0; r < 6; r++) {
        if (roles & p.bb[r]) return "piece bitboards overlap";
        roles |= p.bb[r];
    }
    if (roles != (w | b)) return "piece and colour bitboards disagree";
    if (p.turn > 1 || p.castling > 15) return "bad turn or castling field";
    for (int c = 0; c < 2; c++) {
        const uint64_t s = c ? b : w;
        if (popc64(p.bb[KING] & s) != 1) return "each side needs exactly one king";
        const int pawns = popc64(p.bb[PAWN] & s);
        if (popc64(s) > 16 || pawns > 8) return "too much material";
        const int extra = (popc64(p.bb[QUEEN] & s) > 1 ? popc64(p.bb[QUEEN] & s) - 1 : 0) +
                          (popc64(p.bb[ROOK] & s) > 2 ? popc64(p.bb[ROOK] & s) - 2 : 0) +
                          (popc64(p.bb[BISHOP] & s) > 2 ? popc64(p.bb[BISHOP] & s) - 2 : 0) +
                          (popc64(p.bb[KNIGHT] & s) > 2 ? popc64(p.bb[KNIGHT] & s) - 2 : 0);
        if (extra > 8 - pawns) return "too much material";
    }
    if (p.bb[PAWN] & BACKRANKS) return "pawns on a back rank";
    auto has = [&](int role, uint64_t side, int sq) { return (p.bb[role] & side & (1ULL << sq)) != 0; };
    if ((p.castling & 3) && !has(KING, w, 4)) return "invalid castling rights";
    if (((p.castling & 1) && !has(ROOK, w, 7)) || ((p.castling & 2) && !has(ROOK, w, 0))) return "invalid castling rights";
    if ((p.castling & 12) && !has(KING, b, 60)) return "invalid castling rights";
    if (((p.castling & 4) && !has(ROOK, b, 63)) || ((p.castling & 8) && !has(ROOK, b, 56))) return "invalid castling rights";
    const uint64_t occ = w | b;
    const int ep = raw_ep < 0 ? p.ep : raw_ep, fwd = p.turn ? 8 : -8;   // the pushed pawn stands one rank beyond ep
    if (ep < 64) {
        const uint64_t them = p.turn ? w : b;
        if ((ep >> 3) != (p.turn ? 2 : 5) || (occ & (1ULL << ep)) || (occ & (1ULL << (ep - fwd))) ||
            !(p.bb[PAWN] & them & (1ULL << (ep + fwd))))
            return "invalid en-passant square";
        if (raw_ep < 0 && pseudo_ep(p, ep) != ep) return "en-passant square no pawn can take";
    } else if (ep != 64) {
        return "invalid en-passant square";
    }
    if (raw_ep >= 0 && p.ep != pseudo_ep(p, raw_ep)) return "en-passant square not the pseudo-legal one";
    auto attackers_of = [&](int color, uint64_t o) {   // pieces of !color attacking color's king (occupancy o)
        const uint64_t kbb = p.bb[KING] & (color ? b : w), th = color ? w : b, e = ~o;
        return (pawn_att(color, kbb) & p.bb[PAWN] & th) | (knight_att(kbb) & p.bb[KNIGHT] & th) |
               (king_att(kbb) & p.bb[KING] & th) | (bishop_att(kbb, e) & (p.bb[BISHOP] | p.bb[QUEEN]) & th) |
               (rook_att(kbb, e) & (p.bb[ROOK] | p.bb[QUEEN]) & th);
    };
    if (attackers_of(p.turn ^ 1, occ)) return "the side not to move is in check";
    const uint64_t checkers = attackers_of(p.turn, occ);
    const int ksq = ctz64(p.bb[KING] & (p.turn ? b : w));
    // two checkers on one line through the king (or more than two) cannot come from one move
    if (popc64(checkers) > 2 || (popc64(checkers) == 2 && aligned3(ctz64(checkers), ksq, 63 - clz64(checkers))))
        return "impossible check";
    if (ep < 64 && checkers) {   // the double push must have given the check: the pushed pawn is the one
        const int to = ep + fwd, from = ep - fwd;   // checker, or it uncovered one slider's
        const uint64_t before = (occ & ~(1ULL << to)) | (1ULL << from);
        if (popc64(checkers) > 1 || ((checkers & ~(1ULL << to)) && attackers_of(p.turn, before)))
            return "impossible check (en passant)";
    }
    Pos q = p;
    bool chk;
    if (finalize(q, &chk) > 218) return "more than 218 legal moves";
    return nullptr;
}

AZ_HD Pos startpos() {
    Pos p;
    p.bb[PAWN] = 0x00FF00000000FF00ULL;
    p.bb[KNIGHT] = 0x4200000000000042ULL;
    p.bb[BISHOP] = 0x2400000000000024ULL;
    p.bb[ROOK] = 0x8100000000000081ULL;
    p.bb[QUEEN] = 0x0800000000000008ULL;
    p.bb[KING] = 0x1000000000000010ULL;
    p.bb[WHITE_BB] = 0xFFFFULL;
    p.bb[BLACK_BB] = 0xFFFFULL << 48;
    p.turn = 0; p.castling = 15; p.ep = 64; p.flags = 0; p.halfmoves = 0; p.fullmoves = 1;
    p.rep_key = 0;
    bool chk;
    finalize(p, &chk);
    return p;
}

// outcome() given the legal move count: ONGOING / DRAW / WHITE_WINS / BLACK_WINS
AZ_HD int outcome(const Pos& p, int nlegal, bool in_check) {
    if (nlegal == 0) return in_check ? (p.turn == 0 ? BLACK_WINS : WHITE_WINS) : DRAW;
    if (insufficient_material(p)) return DRAW;
    return ONGOING;
}

// to_tensor (chess.rs:191-245) for one (plane, square) in the side-to-move frame
AZ_HD float plane_value(const Pos& p, int plane, int sq /* rank'*8+file */) {
    const int us = p.turn;
    const int rank = sq >> 3, file = sq & 7;
    const int real = (us ? 7 - rank : rank) * 8 + file;
    const uint64_t m = 1ULL << real;
    if (plane < 12) {
        const int color = plane < 6 ? us : us ^ 1;
        return (role_bb(p, plane % 6) & side_bb(p, color) & m) ? 1.0f : 0.0f;
    }
    switch (plane) {
        case 12: return (p.castling & (us == 0 ? 1 : 4)) ? 1.0f : 0.0f;
        case 13: return (p.castling & (us == 0 ? 2 : 8)) ? 1.0f : 0.0f;
        case 14: return (p.castling & (us == 0 ? 4 : 1)) ? 1.0f : 0.0f;
        case 15: return (p.castling & (us == 0 ? 8 : 2)) ? 1.0f : 0.0f;
        case 16: return p.ep == real ? 1.0f : 0.0f;
        case 17: return (float)p.halfmoves / (float)NUM_HALFMOVES;
        default: return (float)p.fullmoves / (float)NUM_FULLMOVES;
    }
}

}  // namespace azc

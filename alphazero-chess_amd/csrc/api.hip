// api.hip -- C-ABI entry points of libaz for the rules/codec, GameState and network.
// (search / self-play entry points live in search.hip)
#include <string.h>

#include <cstdio>
#include <string>
#include <vector>

#include "az_internal.h"

namespace azi {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
int fail(const std::string& m) { g_err = m; return -1; }
}  // namespace azi

using namespace azi;

namespace {
inline const azc::Pos& P(const az_pos* p) { return *reinterpret_cast<const azc::Pos*>(p); }
inline azc::Pos& P(az_pos* p) { return *reinterpret_cast<azc::Pos*>(p); }

struct VecSink {
    int32_t* out; int cap; int n;
    void operator()(int idx) {
        // under-promotions: the reference's `moves` holds the queen index 4 times (tree.rs:86-89)
        const int reps = (idx & azc::PROMO_FLAG) ? 4 : 1;
        for (int r = 0; r < reps; r++) { if (n < cap) out[n] = idx & azc::IDX_MASK; n++; }
    }
};
}  // namespace

struct az_game {
    std::vector<azc::Pos> hist;     // every position reached, startpos first (pos_count, chess.rs:16)
    std::vector<int32_t> moves;
};

extern "C" {

const char* az_last_error(void) { return g_err.c_str(); }
int az_version(void) { return 1; }

int az_device_count(int* n) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    if (n) *n = c;
    return 0;
}

int az_device_synchronize(int device) {
    AZ_HIP(hipSetDevice(device));
    AZ_HIP(hipDeviceSynchronize());
    return 0;
}

int az_pos_startpos(az_pos* out) {
    if (!out) return fail("null");
    P(out) = azc::startpos();
    return 0;
}

int az_pos_from_fen(const char* fen, az_pos* out) {
    if (!fen || !out) return fail("null");
    azc::Pos p;
    memset(&p, 0, sizeof(p));
    const char* c = fen;
    int r = 7, f = 0;
    for (; *c && *c != ' '; c++) {
        if (*c == '/') { r--; f = 0; continue; }
        if (*c >= '1' && *c <= '8') { f += *c - '0'; continue; }
        const char* roles = "pnbrqk";
        const char* q = strchr(roles, *c | 32);
        if (!q || r < 0 || f > 7) return fail(std::string("bad FEN board: ") + fen);
        const int sq = r * 8 + f;
        p.bb[q - roles] |= 1ULL << sq;
        p.bb[(*c >= 'a') ? azc::BLACK_BB : azc::WHITE_BB] |= 1ULL << sq;
        f++;
    }
    if (*c != ' ') return fail("bad FEN");
    c++;
    p.turn = *c == 'b' ? 1 : 0;
    while (*c && *c != ' ') c++;
    while (*c == ' ') c++;
    p.castling = 0;
    for (; *c && *c != ' '; c++) {
        if (*c == 'K') p.castling |= 1;
        if (*c == 'Q') p.castling |= 2;
        if (*c == 'k') p.castling |= 4;
        if (*c == 'q') p.castling |= 8;
    }
    auto has = [&](int role, int color, int sq) {
        return (p.bb[role] & p.bb[azc::WHITE_BB + color] & (1ULL << sq)) != 0;
    };
    if (!has(azc::KING, 0, 4)) p.castling &= ~3;
    if (!has(azc::ROOK, 0, 7)) p.castling &= ~1;
    if (!has(azc::ROOK, 0, 0)) p.castling &= ~2;
    if (!has(azc::KING, 1, 60)) p.castling &= ~12;
    if (!has(azc::ROOK, 1, 63)) p.castling &= ~4;
    if (!has(azc::ROOK, 1, 56)) p.castling &= ~8;
    while (*c == ' ') c++;
    int ep = 64;
    if (*c && *c != '-') {
        if (c[0] < 'a' || c[0] > 'h' || c[1] < '1' || c[1] > '8') return fail("bad FEN ep");
        ep = (c[1] - '1') * 8 + (c[0] - 'a');
        c += 2;
    } else if (*c) {
        c++;
    }
    int hm = 0, fm = 1;
    if (*c) sscanf(c, " %d %d", &hm, &fm);
    p.halfmoves = (uint16_t)hm;
    p.fullmoves = (uint16_t)(fm < 1 ? 1 : fm);
    // shakmaty validates the ep square as written (EnPassant::from_setup) and keeps the
    // pseudo-legal one: a structurally invalid square is refused, a valid one no pawn can take is
    // dropped.  Validated before finalize, whose move generator assumes one king per side
    p.ep = azc::pseudo_ep(p, ep);
    if (const char* why = azc::setup_error(p, ep)) return fail(std::string("FEN rejected (") + why + "): " + fen);
    bool chk;
    azc::finalize(p, &chk);
    P(out) = p;
    return 0;
}

int az_pos_to_fen(const az_pos* pp, char* buf, int cap) {
    if (!pp || !buf) return fail("null");
    const azc::Pos& p = P(pp);
    std::string s;
    for (int r = 7; r >= 0; r--) {
        int empty = 0;
        for (int f = 0; f < 8; f++) {
            const int sq = r * 8 + f;
            const int role = azc::piece_role_at(p, sq);
            if (role < 0) { empty++; continue; }
            if (empty) { s += (char)('0' + empty); empty = 0; }
            char ch = "PNBRQK"[role];
            if (p.bb[azc::BLACK_BB] & (1ULL << sq)) ch = (char)(ch | 32);
            s += ch;
        }
        if (empty) s += (char)('0' + empty);
        if (r) s += '/';
    }
    s += p.turn ? " b " : " w ";
    if (!p.castling) s += '-';
    if (p.castling & 1) s += 'K';
    if (p.castling & 2) s += 'Q';
    if (p.castling & 4) s += 'k';
    if (p.castling & 8) s += 'q';
    s += ' ';
    if (p.ep >= 64) s += '-';
    else { s += (char)('a' + (p.ep & 7)); s += (char)('1' + (p.ep >> 3)); }
    s += " " + std::to_string(p.halfmoves) + " " + std::to_string(p.fullmoves);
    if ((int)s.size() + 1 > cap) return fail("buffer too small");
    memcpy(buf, s.c_str(), s.size() + 1);
    return (int)s.size();
}

uint64_t az_pos_fen_key(const az_pos* p) { return p ? azc::fen_key(P(p)) : 0; }

int az_pos_legal_indices(const az_pos* p, int32_t* out, int cap) {
    if (!p) return fail("null");
    VecSink s{out, out ? cap : 0, 0};
    bool chk, lep;
    azc::gen_legal(P(p), s, &chk, &lep);
    return s.n;
}

int az_pos_play_index(const az_pos* p, int32_t index, az_pos* child) {
    if (!p || !child) return fail("null");
    if (index < 0 || index >= AZ_ACTION_SPACE) return 0;
    int32_t lst[AZ_MAX_MOVES];
    const int n = az_pos_legal_indices(p, lst, AZ_MAX_MOVES);
    bool ok = false;
    for (int i = 0; i < n; i++) ok |= lst[i] == index;
    if (!ok) return 0;
    azc::Pos c = azc::play_index(P(p), index);
    bool chk;
    azc::finalize(c, &chk);
    P(child) = c;
    return 1;
}

int az_move_to_index(int from, int to, int turn) { return azc::move_index(from, to, turn); }

int az_pos_outcome(const az_pos* p) {
    if (!p) return fail("null");
    azc::NullSink ns;
    bool chk, lep;
    const int n = azc::gen_legal(P(p), ns, &chk, &lep);
    return azc::outcome(P(p), n, chk);
}

int az_pos_encode(const az_pos* p, float* out) {
    if (!p || !out) return fail("null");
    for (int pl = 0; pl < 19; pl++)
        for (int sq = 0; sq < 64; sq++) out[pl * 64 + sq] = azc::plane_value(P(p), pl, sq);
    return 0;
}

// ---------------- GameState (chess.rs:13-63) ----------------
int az_game_create(az_game** out) {
    if (!out) return fail("null");
    az_game* g = new az_game();
    g->hist.push_back(azc::startpos());
    *out = g;
    return 0;
}
int az_game_clone(const az_game* g, az_game** out) {
    if (!g || !out) return fail("null");
    *out = new az_game(*g);
    return 0;
}
int az_game_destroy(az_game* g) { delete g; return 0; }
int az_game_position(const az_game* g, az_pos* out) {
    if (!g || !out) return fail("null");
    P(out) = g->hist.back();
    return 0;
}
int az_game_history(const az_game* g, int32_t* moves, int cap) {
    if (!g) return fail("null");
    const int n = (int)g->moves.size();
    for (int i = 0; i < n && i < cap && moves; i++) moves[i] = g->moves[i];
    return n;
}
int az_game_play(az_game* g, int32_t index) {
    if (!g) return fail("null");
    const azc::Pos cur = g->hist.back();
    az_pos child;
    if (!az_pos_play_index(reinterpret_cast<const az_pos*>(&cur), index, &child)) return AZ_ILLEGAL;
    const azc::Pos& c = P(&child);
    g->hist.push_back(c);
    g->moves.push_back(index);
    azc::NullSink ns;
    bool chk, lep;
    const int n = azc::gen_legal(c, ns, &chk, &lep);
    const int oc = azc::outcome(c, n, chk);
    if (oc != azc::ONGOING) return oc;
    int count = 0;
    for (size_t i = 0; i < g->hist.size(); i++) count += azc::chess_eq(g->hist[i], c) ? 1 : 0;
    if (count < azc::REPETITIONS && c.halfmoves < azc::NUM_HALFMOVES && c.fullmoves < azc::NUM_FULLMOVES)
        return AZ_ONGOING;
    return AZ_DRAW;
}

// ---------------- network ----------------
size_t az_net_num_params(int B, int F) {
    size_t n = (size_t)F * 19 * 9 + F + 4 * (size_t)F;
    n += (size_t)B * 2 * ((size_t)F * F * 9 + F + 4 * (size_t)F);
    n += 32 * (size_t)F + 32 + 4 * 32;
    n += 64 * 32 + 64;
    n += 8 * (size_t)F + 8 + 4 * 8;
    n += 512 * 64 + 64 + 64 + 1;
    return n;
}

int az_net_create(const az_net_desc* d, const float* w, size_t n, int device, az_net** out) {
    if (!d || !w || !out) return fail("null argument");
    NetDev* dev = nullptr;
    const int rc = net_create(d, w, n, device, &dev);
    if (rc) return rc;
    *out = new az_net{dev};
    return 0;
}

int az_net_destroy(az_net* net) {
    if (!net) return 0;
    net_destroy(net->dev);
    delete net;
    return 0;
}

int az_net_tower_kernel(az_net* net, char* out, int cap) {
    if (!net || !out || cap <= 0) return fail("null argument");
    const NetDev* n = net->dev;
    std::string k;
    const std::string F = std::to_string(n->filters);
    if (!(n->fused && tower_supported(n))) k = "conv3x3_kernel (per layer) + heads_kernel";
    else if (n->dtype == AZ_DTYPE_BF16) k = "tower_kernel<" + F + "> (bf16, direct 3x3)";
    else if (wino_supported(n)) k = "tower32w_kernel<" + F + "> (f32, Winograd F(2x2,3x3) residual convs)";
    else k = "tower32_kernel<" + F + "> (f32, direct 3x3)";
    snprintf(out, (size_t)cap, "%s", k.c_str());
    return 0;
}

static int ensure_scratch(NetDev* n, int rows) {
    if (rows <= n->scratch_rows) return 0;
    (void)hipFree(n->x); (void)hipFree(n->h); (void)hipFree(n->planes);
    n->x = n->h = n->planes = nullptr;
    const size_t ab = act_bytes(n->dtype);
    AZ_HIP(hipMalloc(&n->x, (size_t)rows * 64 * n->filters * ab));
    AZ_HIP(hipMalloc(&n->h, (size_t)rows * 64 * n->filters * ab));
    AZ_HIP(hipMalloc(&n->planes, (size_t)rows * 64 * 32 * ab));
    n->scratch_rows = rows;
    return 0;
}

int az_net_forward_device(az_net* net, const float* d_planes, int rows, float* d_policy, float* d_value,
                          void* stream) {
    if (!net) return fail("null net");
    if (rows <= 0) return 0;
    NetDev* n = net->dev;
    AZ_HIP(hipSetDevice(n->device));
    hipStream_t st = stream ? (hipStream_t)stream : n->stream;
    int rc = ensure_scratch(n, rows);
    if (!rc) rc = net_planes_from_host_layout(n, d_planes, rows, n->planes, st);
    if (n->fused && tower_supported(n)) {
        if (!rc) rc = tower_forward(n, n->planes, nullptr, rows, d_policy, d_value, nullptr, st);
        return rc;
    }
    if (!rc) rc = net_tower(n, n->planes, nullptr, rows, n->x, n->h, st, nullptr, nullptr);
    if (!rc) rc = net_heads_dense(n, n->x, rows, d_policy, d_value, st);
    return rc;
}

int az_net_forward(az_net* net, const float* planes, int rows, float* policy, float* value) {
    if (!net || !planes || !policy || !value) return fail("null argument");
    if (rows <= 0) return 0;
    NetDev* n = net->dev;
    AZ_HIP(hipSetDevice(n->device));
    if (rows > n->io_rows) {
        (void)hipFree(n->d_in); (void)hipFree(n->d_pol); (void)hipFree(n->d_val);
        AZ_HIP(hipMalloc(&n->d_in, (size_t)rows * 19 * 64 * 4));
        AZ_HIP(hipMalloc(&n->d_pol, (size_t)rows * 4096 * 4));
        AZ_HIP(hipMalloc(&n->d_val, (size_t)rows * 4));
        n->io_rows = rows;
    }
    AZ_HIP(hipMemcpyAsync(n->d_in, planes, (size_t)rows * 19 * 64 * 4, hipMemcpyHostToDevice, n->stream));
    int rc = az_net_forward_device(net, n->d_in, rows, n->d_pol, n->d_val, n->stream);
    if (rc) return rc;
    AZ_HIP(hipMemcpyAsync(policy, n->d_pol, (size_t)rows * 4096 * 4, hipMemcpyDeviceToHost, n->stream));
    AZ_HIP(hipMemcpyAsync(value, n->d_val, (size_t)rows * 4, hipMemcpyDeviceToHost, n->stream));
    AZ_HIP(hipStreamSynchronize(n->stream));
    return 0;
}

}  // extern "C"

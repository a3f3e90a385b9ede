// az_internal.h -- shared definitions of libaz's translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/az.h"
#include "chess.h"

static_assert(sizeof(az_pos) == 80, "az_pos layout");
static_assert(sizeof(azc::Pos) == sizeof(az_pos), "Pos == az_pos");

#ifndef AZ_WINOGRAD_DEFAULT
#define AZ_WINOGRAD_DEFAULT 1
#endif

namespace azi {

void set_error(const std::string& msg);
int fail(const std::string& msg);

#define AZ_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ::azi::fail(std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

// ---------------- loads of state another launch rewrote ----------------
// A load at a provably wave-uniform address compiles to s_load, which goes through the scalar
// data cache; measured on MI355X (round 2): that cache can still hold the line a previous launch
// of the stream read, so vector stores made in between are not seen (k_expand read stale leaf
// records).  Engine state that launches hand to each other (batch counters, row -> game maps,
// per-game records) is therefore read through vector loads: load_fresh for a single counter,
// vgpr_index for an index that would otherwise make every load behind it scalar.
__device__ __forceinline__ int load_fresh(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int vgpr_index(int i) {
    asm volatile("" : "+v"(i));
    return i;
}

// ---------------- search tree records (HBM, struct-of-arrays per game) ----------------
struct Node {            // 16 B
    uint32_t edge_begin; // first edge (game-relative)
    uint16_t nedges;     // distinct legal move indices
    uint16_t depth;      // root = 0
    uint32_t nsum;       // sum of child visits (tree.rs:121 minus the +1)
    int32_t parent;
};
struct Edge {            // 16 B, one dwordx4 per lane in the select walk
    float P;             // prior (policy[i], noised at roots)
    float W;             // scores[i]
    uint16_t N;          // visits[i]
    uint16_t idx;        // move index | PROMO_FLAG
    int32_t child;       // node id, or CHILD_*
};
static_assert(sizeof(Node) == 16 && sizeof(Edge) == 16, "tree record layout");
enum { CHILD_NONE = -1, CHILD_DRAW = -2, CHILD_WIN = -3 };
enum { LEAF_EVAL = 0, LEAF_DRAW = 1, LEAF_WIN = 2, LEAF_CACHED = 3 };
constexpr int MAX_EDGES = 224;     // >= 218 legal moves
constexpr int HMAX = 512;          // game history cap (200 fullmoves -> <= 400 plies)

struct StepRec {                   // device -> host self-play record, 1024 B
    int32_t game_id;
    int16_t ply, action, depth, nvis, kind, result;   // kind 0 = step, 1 = game end
    int16_t end_fullmoves, pad;
    int32_t pad2;
    azc::Pos pos;
    uint16_t vis_idx[MAX_EDGES];
    uint16_t vis_n[MAX_EDGES];
    uint8_t tail[1024 - 24 - 80 - 4 * MAX_EDGES];
};
static_assert(sizeof(StepRec) == 1024, "StepRec");

struct Counters {                  // device-side statistics
    unsigned long long sims, evals, terminal, games_finished, moves, depth_sum, select_bytes, cache_hits;
    int batch_count[2];            // rows of simulation step i in [i & 1]; the backup of step i
                                   // reads and clears it (no reset launch, and the fused step
                                   // kernel allocates step i rows while it backs up step i - 1)
    int rec_count;
    int next_game_id;
    int log_count;
    int log_prior_count;
    int overflow;
    int pad[1];
};

// everything the tree kernels need, passed by value
struct Engine {
    int G, S, NMAX, EMAX, PMAX;
    float c_puct, dir_alpha, dir_eps;
    int temp_moves, noise, continuous;
    unsigned long long seed;
    Node* nodes;          // [G][NMAX]
    azc::Pos* npos;       // [G][NMAX]
    Edge* edges;          // [G][EMAX]
    uint32_t* child_hdr;  // [G][EMAX]: for an edge whose child is a node, (child's edge_begin << 8) | nedges
    int* node_count; int* edge_count; int* max_depth;
    int* leaf_node; int* leaf_edge; int* leaf_len; int* leaf_kind; int* leaf_row;
    int* path_node; int* path_edge;        // [G][PMAX]
    azc::Pos* hist; int* hist_len;         // [G][HMAX]
    int* game_id; int* ply; int* active;
    int* row_game; int* row_node;          // [G]
    float* value;                          // [G] per batch row
    const float* sqrt_tab;                 // [S + 2]
    Edge* start_edges; int* start_n;       // startpos root template (priors un-noised)
    StepRec* recs; int rec_cap;
    Counters* ctr;
    int* batch_hist;                       // [S] rows evaluated per sim step
    // FEN evaluation cache (tree.rs:214-219): open addressing, CACHE_PROBES linear probes
    int cache_mask;                        // slots - 1 (slots = power of two), -1 = off
    unsigned* c_state;                     // 0 empty, 1 being written, 2 valid
    unsigned long long* c_key;
    azc::Pos* c_pos;
    float* c_value;
    int* c_n;
    float* c_pri;                          // [slots][MAX_EDGES]
    float* cached_value;                   // [G] value of a cache-served leaf
    unsigned long long* g_sims;            // [G] simulations backed up (summed at readout)
    unsigned long long* g_evals;           // [G] network rows of the persistent kernel (summed at readout)
    unsigned long long* g_sel_bytes;       // [G] algorithmic bytes read by k_select
    unsigned long long* trace;             // [G][8] s_memtime phase stamps of k_step (AZ_STEP_TRACE builds only)
    // evaluation log
    int log_cap, log_prior_cap;
    unsigned long long* log_key; float* log_value; int* log_off; int* log_n; int* log_idx; float* log_prior;
};

// ---------------- network ----------------
struct NetDev {
    int blocks = 0, filters = 0, dtype = 0, device = 0;
    std::vector<void*> conv_w;      // swizzled MFMA fragments per conv (1 + 2*blocks)
    std::vector<float*> conv_b;     // folded bias per conv
    std::vector<size_t> conv_bytes; // allocation size of each conv_w (incl. the 8 zero k-steps of prefetch pad)
    std::vector<void*> wino_w;      // f32 F >= 64: Winograd-transformed residual conv weights (tower32w_kernel)
    std::vector<size_t> wino_bytes;
    bool winograd = AZ_WINOGRAD_DEFAULT != 0;   // tower32w_kernel for f32 F >= 64 nets (env AZ_WINOGRAD=0/1)
    float* head = nullptr;          // folded head weights (f32)
    void* head_frag = nullptr;      // 1x1 F->40 head conv as bf16 hi/lo MFMA A-fragments (fused tower)
    void* in_pk32 = nullptr;        // f32 Winograd nets: the input conv's weights with channels 16-18 of 4 taps packed per k-step (tower32w)
    size_t in_pk32_bytes = 0;
    void* head_frag32 = nullptr;    // the same conv as f32 A-fragments of v_mfma_f32_16x16x4_f32 (f32 fused tower)
    size_t head_floats = 0;
    hipStream_t stream = nullptr;
    bool fused = true;              // use tower_forward when supported (AZ_FUSED_TOWER=0 disables)
    // scratch for az_net_forward
    void* x = nullptr; void* h = nullptr; void* planes = nullptr; int scratch_rows = 0;
    float* d_in = nullptr; float* d_pol = nullptr; float* d_val = nullptr; int io_rows = 0;
};

// offsets inside NetDev::head
struct HeadLayout {
    size_t w40, b40, p2w, p2b, l1w, l1b, l2w, l2b, p2f, total;
    __host__ __device__ static HeadLayout make(int F) {
        HeadLayout L;
        L.w40 = 0;                      // [40][F]: policy_conv_1 (32) then value_conv (8), BN folded
        L.b40 = L.w40 + 40 * (size_t)F;
        L.p2w = L.b40 + 40;             // [64][32]
        L.p2b = L.p2w + 64 * 32;
        L.l1w = L.p2b + 64;             // [512][64]
        L.l1b = L.l1w + 512 * 64;
        L.l2w = L.l1b + 64;             // [64]
        L.l2b = L.l2w + 64;
        L.p2f = L.l2b + 4;              // p2w as MFMA A-fragments [cf 4][lane 64][8] (one 32-byte read per lane)
        L.total = L.p2f + 4 * 64 * 8;
        return L;
    }
};

// search-mode output target of the heads / synthetic evaluator
struct SearchOut {
    const Node* nodes; Edge* edges; int NMAX, EMAX;
    const int* row_game; const int* row_node;
    float* value;
    // eval log (may be disabled: log_cap == 0)
    int log_cap, log_prior_cap;
    unsigned long long* log_key; float* log_value; int* log_off; int* log_n; int* log_idx; float* log_prior;
    Counters* ctr;
    const azc::Pos* npos;
};

int net_create(const az_net_desc* d, const float* w, size_t n, int device, NetDev** out);
void net_destroy(NetDev* n);
// planes [rows][64][32] in the net's dtype (device). count may be nullptr (all rows valid).
// ev0/ev1 (optional) bracket the first residual conv launch (timing of one 3x3 FxF conv)
int net_tower(NetDev* n, const void* planes, const int* count, int rows, void* x, void* h, hipStream_t st,
              hipEvent_t ev0, hipEvent_t ev1);
int net_heads_dense(NetDev* n, const void* x, int rows, float* policy, float* value, hipStream_t st);
int net_heads_search(NetDev* n, const void* x, const int* count, int rows, const SearchOut& so, hipStream_t st);
int net_encode_rows(NetDev* n, const azc::Pos* npos, int NMAX, const int* row_game, const int* row_node,
                    const int* count, int rows, void* planes, hipStream_t st);
int synth_eval_rows(const int* count, int rows, const SearchOut& so, hipStream_t st);
int net_planes_from_host_layout(NetDev* n, const float* d_in, int rows, void* planes, hipStream_t st);
// fused tower (tower.hip): input conv + residual tower + heads in one launch (bf16 and f32).
bool tower_supported(const NetDev* n);
bool wino_supported(const NetDev* n);   // f32, F >= 64, Winograd weights built: tower32w_kernel
// persistent per-game simulation kernel (tower.hip, k_sims32w): simulation steps [step0, step1) of
// every game, tree steps and Winograd evaluations in one workgroup per game, all backed up at the end
bool sims_persistent_supported(const NetDev* n);
int sims_persistent(const NetDev* n, const Engine& E, const SearchOut& so, int step0, int step1, hipStream_t st);
int tower_forward(NetDev* n, const void* planes, const int* count, int rows, float* pol, float* val,
                  const SearchOut* so, hipStream_t st);
size_t act_bytes(int dtype);
double net_flop_per_eval(int blocks, int filters);
double net_tower_flop_per_eval(int blocks, int filters);

}  // namespace azi

struct az_net { azi::NetDev* dev; };

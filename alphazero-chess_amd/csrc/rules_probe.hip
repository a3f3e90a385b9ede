// rules_probe.hip -- the device rules path, one item at a time, for parity tests (az_rules_probe).
//
// The search kernels decide legality, outcomes and repetition keys of every new leaf on the GPU
// with their own wave-parallel move generator (search_dev.h leaf_rules / gen_legal_wave), the
// roots with the serial generator (chess.h gen_legal, k_root_setup), and the network sees the
// leaf through the tower's plane staging (chess.h plane_value, stage_planes_f32).  This entry
// runs exactly those device functions on caller-given positions so tests can compare them with
// the oracle's restatement of chess.rs:36-63 / 73-171 / 191-245 on edge positions, perft trees
// and random playouts.  It is a test hook: the engine itself never calls it.
#include <string.h>

#include <vector>

#include "az_internal.h"
#include "search_dev.h"

namespace azi {

struct ProbeOut {
    azc::Pos* child;
    int* moves; int* nmoves;          // gen_legal_wave (leaf expansion), duplicates expanded
    int* root_moves; int* root_n;     // gen_legal (root setup), duplicates expanded
    int* outcome; int* in_check;
    unsigned long long* fen_key;
    float* planes;                    // [n][19][64]
    Edge* scratch;                    // [n][MAX_EDGES]
};

// under-promotions: the reference's `moves` holds the queen-promotion index 4 times (tree.rs:86-89)
__device__ __forceinline__ int expand_dups(const Edge* e, int n, int* out) {
    int k = 0;
    for (int i = 0; i < n; i++) {
        const int idx = e[i].idx & azc::IDX_MASK, reps = (e[i].idx & azc::PROMO_FLAG) ? 4 : 1;
        for (int r = 0; r < reps; r++) if (k < AZ_MAX_MOVES) out[k++] = idx;
    }
    return k;
}

// one wavefront per item, as one game's expansion in k_expand / k_step
__global__ void __launch_bounds__(64) k_rules_probe(const azc::Pos* __restrict__ parent, const int* __restrict__ action,
                                                    int n, ProbeOut o) {
    const int i = vgpr_index(blockIdx.x), lane = threadIdx.x;
    if (i >= n) return;
    const int a = action[i];
    azc::Pos c = parent[i];
    if (a >= 0) c = azc::play_index(c, a);                   // index_to_move + play (chess.rs:118-171, 42)
    Edge* ed = o.scratch + (size_t)i * MAX_EDGES;
    int ne = 0;
    bool chk = false;
    const int res = leaf_rules<1>(c, ed, lane, &ne, nullptr, &chk);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (lane == 0) {
        o.child[i] = c;
        o.outcome[i] = res;
        o.in_check[i] = chk ? 1 : 0;
        o.fen_key[i] = azc::fen_key(c);
        o.nmoves[i] = expand_dups(ed, ne, o.moves + (size_t)i * AZ_MAX_MOVES);
        // the roots' serial generator (k_root_setup), into the same scratch once it has been read
        EdgeSink sink{ed, 0};
        bool rchk, rlep;
        const int rn = azc::gen_legal(c, sink, &rchk, &rlep);
        o.root_n[i] = expand_dups(ed, rn, o.root_moves + (size_t)i * AZ_MAX_MOVES);
    }
    for (int e = lane; e < 19 * 64; e += 64)                 // to_tensor as the towers stage it
        o.planes[(size_t)i * 19 * 64 + e] = azc::plane_value(c, e >> 6, e & 63);
}

}  // namespace azi

using namespace azi;

extern "C" int az_rules_probe(int device, const az_pos* parent, const int32_t* action, int n, az_pos* child,
                              int32_t* moves, int32_t* nmoves, int32_t* root_moves, int32_t* root_n, int32_t* outcome,
                              int32_t* in_check, uint64_t* fen_key, float* planes) {
    if (n < 0 || (n > 0 && (!parent || !action || !child))) return fail("az_rules_probe: null argument");
    if (n == 0) return 0;
    // the kernels only ever play legal moves: refuse anything else here, on the host
    for (int i = 0; i < n; i++) {
        // the device scratch holds MAX_EDGES moves: a parent shakmaty would refuse (many queens,
        // overlapping bitboards, the side not to move in check ...) is refused here too
        if (const char* why = azc::setup_error(*reinterpret_cast<const azc::Pos*>(parent + i)))
            return fail("az_rules_probe: item " + std::to_string(i) + ": parent rejected: " + why);
        if (action[i] < 0) continue;
        int32_t lst[AZ_MAX_MOVES];
        const int nl = az_pos_legal_indices(parent + i, lst, AZ_MAX_MOVES);
        bool ok = false;
        for (int k = 0; k < nl; k++) ok |= lst[k] == action[i];
        if (!ok) return fail("az_rules_probe: item " + std::to_string(i) + ": index " + std::to_string(action[i]) +
                             " is not legal");
    }
    AZ_HIP(hipSetDevice(device));
    hipStream_t st;
    AZ_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<void*> bufs;
    bool oom = false;
    auto dmal = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, bytes < 16 ? 16 : bytes) != hipSuccess) { oom = true; return nullptr; }
        bufs.push_back(p);
        return p;
    };
    const size_t N = (size_t)n;
    azc::Pos* d_par = (azc::Pos*)dmal(N * sizeof(azc::Pos));
    int* d_act = (int*)dmal(N * 4);
    ProbeOut o;
    o.child = (azc::Pos*)dmal(N * sizeof(azc::Pos));
    o.moves = (int*)dmal(N * AZ_MAX_MOVES * 4);
    o.nmoves = (int*)dmal(N * 4);
    o.root_moves = (int*)dmal(N * AZ_MAX_MOVES * 4);
    o.root_n = (int*)dmal(N * 4);
    o.outcome = (int*)dmal(N * 4);
    o.in_check = (int*)dmal(N * 4);
    o.fen_key = (unsigned long long*)dmal(N * 8);
    o.planes = (float*)dmal(N * 19 * 64 * 4);
    o.scratch = (Edge*)dmal(N * MAX_EDGES * sizeof(Edge));
    int rc = oom ? fail("az_rules_probe: hipMalloc failed") : 0;
    if (!rc) {
        auto run = [&]() -> int {
            AZ_HIP(hipMemcpyAsync(d_par, parent, N * sizeof(azc::Pos), hipMemcpyHostToDevice, st));
            AZ_HIP(hipMemcpyAsync(d_act, action, N * 4, hipMemcpyHostToDevice, st));
            k_rules_probe<<<n, 64, 0, st>>>(d_par, d_act, n, o);
            AZ_HIP(hipGetLastError());
            AZ_HIP(hipMemcpyAsync(child, o.child, N * sizeof(azc::Pos), hipMemcpyDeviceToHost, st));
            if (moves) AZ_HIP(hipMemcpyAsync(moves, o.moves, N * AZ_MAX_MOVES * 4, hipMemcpyDeviceToHost, st));
            if (nmoves) AZ_HIP(hipMemcpyAsync(nmoves, o.nmoves, N * 4, hipMemcpyDeviceToHost, st));
            if (root_moves) AZ_HIP(hipMemcpyAsync(root_moves, o.root_moves, N * AZ_MAX_MOVES * 4, hipMemcpyDeviceToHost, st));
            if (root_n) AZ_HIP(hipMemcpyAsync(root_n, o.root_n, N * 4, hipMemcpyDeviceToHost, st));
            if (outcome) AZ_HIP(hipMemcpyAsync(outcome, o.outcome, N * 4, hipMemcpyDeviceToHost, st));
            if (in_check) AZ_HIP(hipMemcpyAsync(in_check, o.in_check, N * 4, hipMemcpyDeviceToHost, st));
            if (fen_key) AZ_HIP(hipMemcpyAsync(fen_key, o.fen_key, N * 8, hipMemcpyDeviceToHost, st));
            if (planes) AZ_HIP(hipMemcpyAsync(planes, o.planes, N * 19 * 64 * 4, hipMemcpyDeviceToHost, st));
            AZ_HIP(hipStreamSynchronize(st));
            return 0;
        };
        rc = run();
    }
    (void)hipStreamSynchronize(st);
    for (void* p : bufs) (void)hipFree(p);
    (void)hipStreamDestroy(st);
    return rc;
}

// tower.hip -- fused residual tower + heads (agent.rs:112-144) in ONE launch per batch.
//
// Each workgroup owns BPB boards for the whole forward pass: their activations x and h
// (NHWC bf16, padded 16-B-slot rows: conflict-free ds_read_b128 for every 3x3 tap) stay
// resident in LDS across the input conv, all 2B residual convs and the heads; only the
// weights stream from L2 (MFMA-fragment-swizzled, one dwordx4 per lane per fragment,
// prefetched two K-steps ahead).  Between layers there is a workgroup barrier, no HBM
// round trip and no kernel boundary.  Per layer per wave: 32 output channels x
// (BPB/WB) boards on v_mfma_f32_16x16x32_bf16 (fp32 accumulate), bias + (residual) +
// ReLU fused into an epilogue that writes bf16 back into LDS.
// The heads run from the same LDS image (f32 VALU), in dense mode (policy[4096],
// value) or in search mode (softmax gathered at the new node's legal edges).
#include <math.h>
#include <string.h>

#include "az_internal.h"

#ifndef AZ_TOWER_WB256
#define AZ_TOWER_WB256 1   // F=256: 8 waves x 2 boards (WB=2, 16 waves, measured 10% slower: spills)
#endif
#ifndef AZ_TOWER_NCO256
#define AZ_TOWER_NCO256 2
#endif
#ifndef AZ_TOWER_PF
#define AZ_TOWER_PF 2      // weight prefetch depth in k-steps (L2 latency cover; 4 measured no faster)
#endif

namespace azi {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

struct TowerArgs {
    const uint4* w[1 + 2 * 40];    // swizzled conv weights (input conv, then conv1/conv2 per block)
    const float* b[1 + 2 * 40];    // folded biases
    const float* head;
    int blocks;
};

// BPB boards per workgroup; NCO 16-channel output fragments per wave; WB board groups.
// waves = (F / (16*NCO)) * WB
template <int F> struct TowerCfg;
template <> struct TowerCfg<256> { static constexpr int BPB = 2, WB = AZ_TOWER_WB256, NCO = AZ_TOWER_NCO256; };
template <> struct TowerCfg<128> { static constexpr int BPB = 4, WB = 1, NCO = 2; };
template <> struct TowerCfg<64> { static constexpr int BPB = 4, WB = 2, NCO = 2; };
template <> struct TowerCfg<32> { static constexpr int BPB = 8, WB = 4, NCO = 2; };

__device__ __forceinline__ float t_wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float t_wave_sum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One 3x3 conv layer LDS -> LDS.  IN: CIN channels, row stride RSI slots; OUT: F channels,
// row stride RSO slots.  Wave (cw, bw) computes channels [32cw, 32cw+32) of boards
// [bw*BPW, (bw+1)*BPW).  RESID: out = relu(conv(in) + bias + out).
template <int NCH> struct RingPF { static constexpr int PF = NCH >= AZ_TOWER_PF ? AZ_TOWER_PF : NCH; };

// Load k-steps [0, PF) of a layer's weight fragments into the ring.
template <int NCH, int F, int NCO>
__device__ __forceinline__ void ring_fill(uint4 (&wr)[RingPF<NCH>::PF][NCO], const uint4* __restrict__ wsw, int cw,
                                          int lane) {
    constexpr int CF = F / 16;
    const uint4* W = wsw + (size_t)(cw * NCO) * 64 + lane;
#pragma unroll
    for (int i = 0; i < RingPF<NCH>::PF; i++)
#pragma unroll
        for (int n = 0; n < NCO; n++) wr[i][n] = W[(size_t)i * CF * 64 + n * 64];
}

// wr: register ring holding this layer's next PF weight k-steps on entry; on exit it holds
// the first PF k-steps of `wnext` (the next layer with the same chunk count), or zeros.
template <int CIN, int RSI, int F, int RSO, int BPW, int NCO, bool RESID>
__device__ __forceinline__ void conv_lds(const char* __restrict__ ldsb, uint4* __restrict__ out_lds, int in_off,
                                         int zero_off, const uint4* __restrict__ wsw, const uint4* __restrict__ wnext,
                                         const float* __restrict__ bias, uint4 (&wr)[RingPF<CIN / 32>::PF][NCO],
                                         int cw, int bw, int lane) {
    constexpr int NCH = CIN / 32;                     // 32-channel K chunks (4 slots)
    constexpr int CF = F / 16;
    constexpr int MF = BPW * 4;
    constexpr int KS = 9 * NCH;
    // weight fragments are prefetched PF k-steps ahead through a register ring; PF divides
    // NCH so the ring slot of every k-step is a compile-time constant
    constexpr int PF = RingPF<NCH>::PF;
    static_assert(NCH % PF == 0, "prefetch depth must divide the chunk count");
    const int h = lane >> 4;
    // accumulators start at the folded bias: no bias adds in the epilogue
    f32x4 acc[MF][NCO];
#pragma unroll
    for (int n = 0; n < NCO; n++) {
        const float4 bn = *reinterpret_cast<const float4*>(bias + cw * 16 * NCO + n * 16 + h * 4);
#pragma unroll
        for (int m = 0; m < MF; m++) acc[m][n] = f32x4{bn.x, bn.y, bn.z, bn.w};
    }
    const uint4* W = wsw + (size_t)(cw * NCO) * 64 + lane;
    // past the last k-step the refills read the next layer (or this layer's zero padding)
    const uint4* Wn = (wnext ? wnext + (size_t)(cw * NCO) * 64 + lane : W + (size_t)KS * CF * 64) - (size_t)KS * CF * 64;
    // B-fragment (activation) reads run LA fragments ahead, across k-step and tap boundaries:
    // the first LA reads of step s+1 are issued inside step s.
    constexpr int LA = 4;
    static_assert(MF % LA == 0, "read-ahead ring must tile the fragment loop");
    auto tap_bases = [&](int tap, int* base) {
        const int dr = tap / 3 - 1, df = tap % 3 - 1;
#pragma unroll
        for (int m = 0; m < MF; m++) {
            const int b = bw * BPW + (m >> 2);
            const int sq = (m & 3) * 16 + (lane & 15);
            const int r = (sq >> 3) + dr, f = (sq & 7) + df;
            const bool ok = (unsigned)r < 8u && (unsigned)f < 8u;
            const int s2 = (r * 8 + f) & 63;
            base[m] = ok ? in_off + ((b * 64 + s2) * RSI + h) * 16 : zero_off + (((s2 * RSI) & 15) + h) * 16;
        }
    };
    int bcur[MF], bnext[MF];
    tap_bases(0, bcur);
    uint4 bq[LA];
#pragma unroll
    for (int m = 0; m < LA; m++) bq[m] = *reinterpret_cast<const uint4*>(ldsb + bcur[m]);
    for (int tap = 0; tap < 9; tap++) {
        tap_bases(tap < 8 ? tap + 1 : 8, bnext);
#pragma unroll
        for (int cc = 0; cc < NCH; cc++) {
            const int ks = tap * NCH + cc;
            uint4 a[NCO];
#pragma unroll
            for (int n = 0; n < NCO; n++) a[n] = wr[cc % PF][n];
            // refill this ring slot with k-step ks+PF (of the next layer once past the end)
            const uint4* Wsrc = (tap == 8 && cc + PF >= NCH) ? Wn : W;
#pragma unroll
            for (int n = 0; n < NCO; n++) wr[cc % PF][n] = Wsrc[(size_t)(ks + PF) * CF * 64 + n * 64];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < MF; m++) {
                const uint4 bv = bq[m % LA];
                if (m + LA < MF) {
                    bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bcur[m + LA] + cc * 64);
                } else if (cc + 1 < NCH) {                   // next k-step, same tap
                    bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bcur[m + LA - MF] + (cc + 1) * 64);
                } else {                                     // first k-step of the next tap
                    bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bnext[m + LA - MF]);
                }
                const bf16x8 Bv = __builtin_bit_cast(bf16x8, bv);
#pragma unroll
                for (int n = 0; n < NCO; n++)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[n]), Bv,
                                                                        acc[m][n], 0, 0, 0);
            }
#pragma unroll
            for (int m = 0; m < MF; m++) {
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, NCO, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int m = 0; m < MF; m++) bcur[m] = bnext[m];
    }
    (void)KS;
    // `in` and `out` are different buffers, so the epilogue needs no barrier before it;
    // the barrier after it publishes `out` to the next layer.
    char* ob = reinterpret_cast<char*>(out_lds);
    typedef __attribute__((ext_vector_type(2))) float f32x2;
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    typedef __attribute__((ext_vector_type(2))) short s16x2;
    const s16x2 z = {0, 0};
#pragma unroll
    for (int n = 0; n < NCO; n++) {
        const int co = cw * 16 * NCO + n * 16 + h * 4;
        // per-lane base; each fragment adds a compile-time offset (ds_write immediate)
        char* lane_base = ob + ((bw * BPW * 64 + (lane & 15)) * RSO + (co >> 3)) * 16 + (co & 7) * 2;
#pragma unroll
        for (int m = 0; m < MF; m++) {
            uint2* dst = reinterpret_cast<uint2*>(lane_base + ((m >> 2) * 64 + (m & 3) * 16) * RSO * 16);
            f32x2 lo = {acc[m][n][0], acc[m][n][1]}, hi = {acc[m][n][2], acc[m][n][3]};
            if constexpr (RESID) {
                const uint2 r = *dst;                       // bf16 -> f32 is a 16-bit shift
                lo += f32x2{__builtin_bit_cast(float, r.x << 16), __builtin_bit_cast(float, r.x & 0xFFFF0000u)};
                hi += f32x2{__builtin_bit_cast(float, r.y << 16), __builtin_bit_cast(float, r.y & 0xFFFF0000u)};
            }
            // round to bf16 (v_cvt_pk_bf16_f32), then ReLU as a signed 16-bit max with 0
            s16x2 q0 = __builtin_bit_cast(s16x2, __builtin_convertvector(lo, bf16x2));
            s16x2 q1 = __builtin_bit_cast(s16x2, __builtin_convertvector(hi, bf16x2));
            q0 = __builtin_elementwise_max(q0, z);
            q1 = __builtin_elementwise_max(q1, z);
            *dst = make_uint2(__builtin_bit_cast(unsigned, q0), __builtin_bit_cast(unsigned, q1));
        }
    }
    __syncthreads();
}

// heads for one board from the LDS image x (bf16, row stride RS slots); 256 threads (t < 256).
template <int F, int RS, bool SEARCH>
__device__ __forceinline__ void heads_lds(const char* __restrict__ xb, float* __restrict__ scratch, int t,
                                          const float* __restrict__ head, bool writer, bool valid, int row,
                                          float* pol_out, float* val_out, const SearchOut& so) {
    // writer: this 256-thread group owns `scratch` (idle groups only join the barriers)
    const HeadLayout L = HeadLayout::make(F);
    float* p1 = scratch;                 // [32][64]
    float* v1 = p1 + 32 * 64;            // [8][64]
    float* lg = v1 + 8 * 64;             // [4096]
    float* red = lg + 4096;              // [256]
    float* stat = red + 256;             // [8]
    const int sq = t & 63;
    const int g = __builtin_amdgcn_readfirstlane(t >> 6);
    if (valid) {
        float acc[10];
#pragma unroll
        for (int j = 0; j < 10; j++) acc[j] = 0.0f;
        const float* w40 = head + L.w40 + (size_t)g * 10 * F;
        const char* xr = xb + sq * RS * 16;
        for (int c8 = 0; c8 < F / 8; c8++) {
            const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xr + c8 * 16);
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const float x = (float)xv[e];
#pragma unroll
                for (int j = 0; j < 10; j++) acc[j] += w40[j * F + c8 * 8 + e] * x;
            }
        }
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const int ch = g * 10 + j;
            const float v = fmaxf(acc[j] + head[L.b40 + ch], 0.0f);
            if (ch < 32) p1[ch * 64 + sq] = v; else v1[(ch - 32) * 64 + sq] = v;
        }
    }
    __syncthreads();
    float mx = -INFINITY;
    if (valid) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int c2 = g * 16 + j;
            float l = 0.0f;
            for (int c1 = 0; c1 < 32; c1++) l += head[L.p2w + c2 * 32 + c1] * p1[c1 * 64 + sq];
            l += head[L.p2b + c2];
            lg[c2 * 64 + sq] = l;
            mx = fmaxf(mx, l);
        }
        const int o = t & 63;
        float a = 0.0f;
        for (int i = g * 128; i < g * 128 + 128; i++) a += v1[i] * head[L.l1w + i * 64 + o];
        red[g * 64 + o] = a;
    }
    mx = t_wave_max(mx);
    if (writer && (t & 63) == 0) stat[g] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(stat[0], stat[1]), fmaxf(stat[2], stat[3]));
    float s = 0.0f;
    if (valid)
        for (int i = t; i < 4096; i += 256) s += expf(lg[i] - mx);
    s = t_wave_sum(s);
    float hv = 0.0f;
    if (writer && t < 64) {
        const float hsum = red[t] + red[64 + t] + red[128 + t] + red[192 + t] + head[L.l1b + t];
        hv = fmaxf(hsum, 0.0f) * head[L.l2w + t];
    }
    __syncthreads();
    if (writer && (t & 63) == 0) stat[4 + g] = s;
    if (writer && t < 64) {
        hv = t_wave_sum(hv);
        if (t == 0) red[0] = tanhf(hv + head[L.l2b]);
    }
    __syncthreads();
    const float sum = stat[4] + stat[5] + stat[6] + stat[7];
    const float value = red[0];
    if (valid) {
        if constexpr (!SEARCH) {
            float* pr = pol_out + (size_t)row * 4096;
            for (int i = t; i < 4096; i += 256) pr[i] = expf(lg[i] - mx) / sum;
            if (t == 0) val_out[row] = value;
        } else {
            const int game = so.row_game[row], node = so.row_node[row];
            const Node nd = so.nodes[(size_t)game * so.NMAX + node];
            Edge* e = so.edges + (size_t)game * so.EMAX + nd.edge_begin;
            for (int i = t; i < nd.nedges; i += 256) {
                const int idx = e[i].idx & azc::IDX_MASK;
                e[i].P = expf(lg[idx] - mx) / sum;
            }
            if (t == 0) so.value[row] = value;
            if (so.log_cap > 0) {
                int* slot = reinterpret_cast<int*>(stat + 8);
                if (t == 0) {
                    const int r = atomicAdd(&so.ctr->log_count, 1);
                    const int po = atomicAdd(&so.ctr->log_prior_count, (int)nd.nedges);
                    slot[0] = (r < so.log_cap && po + nd.nedges <= so.log_prior_cap) ? r : -1;
                    slot[1] = po;
                    if (slot[0] >= 0) {
                        so.log_key[r] = azc::fen_key(so.npos[(size_t)game * so.NMAX + node]);
                        so.log_value[r] = value;
                        so.log_off[r] = po;
                        so.log_n[r] = nd.nedges;
                    }
                }
                // slot[] (thread 0) is read by the caller after the next __syncthreads
            }
        }
    }
}

template <int F, bool SEARCH>
__global__ void __launch_bounds__((F / (16 * TowerCfg<F>::NCO)) * TowerCfg<F>::WB * 64)
tower_kernel(const __bf16* __restrict__ planes, TowerArgs ta, const int* __restrict__ count_ptr, int rows,
             float* __restrict__ pol_out, float* __restrict__ val_out, SearchOut so) {
    constexpr int BPB = TowerCfg<F>::BPB, WB = TowerCfg<F>::WB, BPW = BPB / WB, NCO = TowerCfg<F>::NCO;
    constexpr int NCW = F / (16 * NCO);
    constexpr int NT = NCW * WB * 64;
    constexpr int RSF = F / 8 + 2, RSI = 32 / 8 + 2;
    constexpr int XSZ = BPB * 64 * RSF;               // slots per activation buffer
    constexpr int ZN = 16 + F / 8;
    constexpr int HEADS_FLOATS = 32 * 64 + 8 * 64 + 4096 + 256 + 16;
    constexpr int PAR = NT / 256 < BPB ? NT / 256 : BPB;   // boards whose heads run concurrently
    static_assert(NT % 256 == 0, "heads need 256-thread groups");
    static_assert(PAR * HEADS_FLOATS * 4 <= XSZ * 16, "heads scratch must fit in h");
    __shared__ __attribute__((aligned(16))) uint4 lds[2 * XSZ + ZN];
    const int count = count_ptr ? min(*count_ptr, rows) : rows;
    const int row0 = blockIdx.x * BPB;
    if (row0 >= count) return;
    const int nb = min(BPB, count - row0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cw = w % NCW, bw = w / NCW;
    uint4* X = lds;
    uint4* H = lds + XSZ;
    const int zero_off = 2 * XSZ * 16;
    const char* ldsb = reinterpret_cast<const char*>(lds);

    // stage the input planes [row][64][32] into H with row stride RSI
    const uint4* src = reinterpret_cast<const uint4*>(planes) + (size_t)row0 * 64 * 4;
    for (int c = tid; c < BPB * 64 * 4; c += NT) {
        const int rowi = c >> 2, slot = c & 3;
        H[rowi * RSI + slot] = rowi < nb * 64 ? src[c] : make_uint4(0, 0, 0, 0);
    }
    for (int c = tid; c < ZN; c += NT) lds[2 * XSZ + c] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    {
        uint4 wr0[RingPF<1>::PF][NCO];
        ring_fill<1, F, NCO>(wr0, ta.w[0], cw, lane);
        conv_lds<32, RSI, F, RSF, BPW, NCO, false>(ldsb, X, XSZ * 16, zero_off, ta.w[0], nullptr, ta.b[0], wr0, cw,
                                                   bw, lane);
    }
    uint4 wr[RingPF<F / 32>::PF][NCO];
    if (ta.blocks > 0) ring_fill<F / 32, F, NCO>(wr, ta.w[1], cw, lane);
    for (int b = 0; b < ta.blocks; b++) {
        const uint4* after = b + 1 < ta.blocks ? ta.w[3 + 2 * b] : nullptr;
        conv_lds<F, RSF, F, RSF, BPW, NCO, false>(ldsb, H, 0, zero_off, ta.w[1 + 2 * b], ta.w[2 + 2 * b],
                                                  ta.b[1 + 2 * b], wr, cw, bw, lane);
        conv_lds<F, RSF, F, RSF, BPW, NCO, true>(ldsb, X, XSZ * 16, zero_off, ta.w[2 + 2 * b], after, ta.b[2 + 2 * b],
                                                 wr, cw, bw, lane);
    }
    // heads: 256-thread groups, PAR boards at a time, scratch in H
    const int grp = tid >> 8, t = tid & 255;
    float* scratch = reinterpret_cast<float*>(H) + (grp < PAR ? grp : 0) * HEADS_FLOATS;
    for (int b0 = 0; b0 < BPB; b0 += PAR) {
        const int b = b0 + grp;
        const bool valid = grp < PAR && b < nb;
        heads_lds<F, RSF, SEARCH>(ldsb + (size_t)(b < BPB ? b : 0) * 64 * RSF * 16, scratch, t, ta.head, grp < PAR,
                                  valid, row0 + b, pol_out, val_out, so);
        __syncthreads();
        if constexpr (SEARCH) {
            if (valid && so.log_cap > 0) {
                const int* slot = reinterpret_cast<const int*>(scratch + 32 * 64 + 8 * 64 + 4096 + 256 + 8);
                if (slot[0] >= 0) {
                    const int game = so.row_game[row0 + b], node = so.row_node[row0 + b];
                    const Node nd = so.nodes[(size_t)game * so.NMAX + node];
                    const Edge* e = so.edges + (size_t)game * so.EMAX + nd.edge_begin;
                    for (int i = t; i < nd.nedges; i += 256) {
                        so.log_idx[slot[1] + i] = e[i].idx & azc::IDX_MASK;
                        so.log_prior[slot[1] + i] = e[i].P;
                    }
                }
            }
        }
        __syncthreads();
    }
}

bool tower_supported(const NetDev* n) {
    return n->dtype == AZ_DTYPE_BF16 && n->blocks <= 40 &&
           (n->filters == 256 || n->filters == 128 || n->filters == 64 || n->filters == 32);
}

int tower_forward(NetDev* n, const void* planes, const int* count, int rows, float* pol, float* val,
                  const SearchOut* so, hipStream_t st) {
    if (rows <= 0) return 0;
    if (!tower_supported(n)) return fail("fused tower: unsupported net");
    TowerArgs ta;
    memset(&ta, 0, sizeof(ta));
    for (int i = 0; i < 1 + 2 * n->blocks; i++) {
        ta.w[i] = reinterpret_cast<const uint4*>(n->conv_w[i]);
        ta.b[i] = n->conv_b[i];
    }
    ta.head = n->head;
    ta.blocks = n->blocks;
    SearchOut dummy;
    memset(&dummy, 0, sizeof(dummy));
    const SearchOut& s = so ? *so : dummy;
#define AZ_TOWER(FF)                                                                                           \
    if (n->filters == FF) {                                                                                    \
        constexpr int BPB = TowerCfg<FF>::BPB;                                                                 \
        constexpr int NT = (FF / (16 * TowerCfg<FF>::NCO)) * TowerCfg<FF>::WB * 64;                            \
        const int grid = (rows + BPB - 1) / BPB;                                                               \
        if (so) tower_kernel<FF, true><<<grid, NT, 0, st>>>((const __bf16*)planes, ta, count, rows, pol, val, s); \
        else tower_kernel<FF, false><<<grid, NT, 0, st>>>((const __bf16*)planes, ta, count, rows, pol, val, s);  \
        return hipGetLastError() == hipSuccess ? 0 : fail("tower launch failed");                              \
    }
    AZ_TOWER(256) AZ_TOWER(128) AZ_TOWER(64) AZ_TOWER(32)
#undef AZ_TOWER
    return fail("fused tower: unsupported filters");
}

}  // namespace azi

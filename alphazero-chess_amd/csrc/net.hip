// net.hip -- AlphaZero network (agent.rs:11-145) on gfx950.
//
// Layout in HBM: activations NHWC [row][64 squares][C] in the compute dtype (bf16 or f32),
// square = rank'*8 + file in the side-to-move frame (chess.rs:191-245).
// conv3x3_kernel: implicit GEMM on MFMA. One workgroup = BPB boards (M = 64*BPB squares)
// x all output channels; wave w owns 32 output channels.  The boards' input tile is staged
// once into LDS (XOR-swizzled 16-B slots, plus one zero row that out-of-board taps read);
// the 9 taps are shifted LDS reads, so K = 9*Cin never touches HBM twice.  Weights are
// pre-swizzled on the host into per-lane MFMA fragments (1 KiB contiguous per fragment,
// one coalesced dwordx4 per lane) and prefetched one K-step ahead from L2.
// Operands: A = weights (16 out-channels x K), B = activations (K x 16 squares), so each
// lane's accumulator holds 4 consecutive channels of one square (8/16-B NHWC stores).
//   bf16: v_mfma_f32_16x16x32_bf16, fp32 accumulate, bf16 activations.
//   f32 : v_mfma_f32_16x16x4_f32 (exact f32 FMA chain), f32 activations.
// BatchNorm (inference, running stats) is folded into conv weight/bias at load time;
// bias + residual + ReLU are fused into the conv epilogue.
// heads_kernel: policy head (1x1 F->32, ReLU, 1x1 32->64, softmax over 4096) and value
// head (1x1 F->8, ReLU, Linear 512->64, ReLU, Linear 64->1, tanh) fused per board; in
// search mode only the legal entries of the softmax leave the kernel (written straight
// into the new node's edge priors).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "az_internal.h"

namespace azi {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

template <typename T> struct DTraits;
template <> struct DTraits<__bf16> { static constexpr int CH_SLOT = 8; static constexpr int CHUNK = 32; };
template <> struct DTraits<float> { static constexpr int CH_SLOT = 4; static constexpr int CHUNK = 16; };

template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }

size_t act_bytes(int dtype) { return dtype == AZ_DTYPE_BF16 ? 2 : 4; }

double net_tower_flop_per_eval(int B, int F) {
    return 2.0 * 64.0 * (171.0 * F + 18.0 * B * (double)F * F);
}
double net_flop_per_eval(int B, int F) {
    return 2.0 * 64.0 * (171.0 * F + 18.0 * B * (double)F * F + 40.0 * F + 2048.0) + 2.0 * (32768.0 + 64.0);
}

// ------------------------------------------------------------------ conv 3x3
template <int CIN, int COUT, int BPB, typename T, bool RESID>
__global__ void __launch_bounds__(COUT * 2)
conv3x3_kernel(const T* __restrict__ in, T* __restrict__ out, const void* __restrict__ wsw,
               const float* __restrict__ bias, const int* __restrict__ count_ptr, int rows) {
    constexpr int NT = COUT * 2;                      // COUT/32 waves
    constexpr int CHS = DTraits<T>::CH_SLOT;          // channels per 16-B slot
    constexpr int NSLOT = CIN / CHS;
    constexpr int RS = NSLOT + 2;                     // padded row stride (slots): conflict-free ds_read_b128
    constexpr int CHUNK = DTraits<T>::CHUNK;          // channels per K-chunk (4 slots)
    constexpr int NCH = CIN / CHUNK;
    constexpr int CF = COUT / 16;
    constexpr int MF = BPB * 4;                       // 16-square fragments per block
    constexpr int ZB = BPB * 64 * RS;                 // zero region (read by off-board taps)
    constexpr int ZN = 16 + NSLOT;
    __shared__ __attribute__((aligned(16))) uint4 lds[ZB + ZN];

    const int count = count_ptr ? min(load_fresh(count_ptr), rows) : rows;
    const int row0 = blockIdx.x * BPB;
    if (row0 >= count) return;
    const int nb = min(BPB, count - row0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

    // stage the boards into padded rows (missing boards and the zero region are zero)
    const uint4* src = reinterpret_cast<const uint4*>(in) + (size_t)row0 * 64 * NSLOT;
    for (int c = tid; c < BPB * 64 * NSLOT; c += NT) {
        const int rowi = c / NSLOT, slot = c - rowi * NSLOT;
        lds[rowi * RS + slot] = rowi < nb * 64 ? src[c] : make_uint4(0, 0, 0, 0);
    }
    for (int c = tid; c < ZN; c += NT) lds[ZB + c] = make_uint4(0, 0, 0, 0);
    __syncthreads();

    f32x4 acc[MF][2];
#pragma unroll
    for (int m = 0; m < MF; m++) { acc[m][0] = f32x4{0, 0, 0, 0}; acc[m][1] = f32x4{0, 0, 0, 0}; }

    const uint4* W = reinterpret_cast<const uint4*>(wsw) + (size_t)(w * 2) * 64 + lane;
    const int h = lane >> 4;
    // weight fragments: register prefetch one k-step ahead (the buffer is padded by one k-step)
    uint4 a0 = W[0], a1 = W[64];
    const char* ldsb = reinterpret_cast<const char*>(lds);

    for (int tap = 0; tap < 9; tap++) {
        const int dr = tap / 3 - 1, df = tap % 3 - 1;
        int base[MF];
#pragma unroll
        for (int m = 0; m < MF; m++) {
            const int b = m >> 2;
            const int sq = (m & 3) * 16 + (lane & 15);
            const int r = (sq >> 3) + dr, f = (sq & 7) + df;
            const bool ok = (unsigned)r < 8u && (unsigned)f < 8u;
            const int s2 = (r * 8 + f) & 63;
            // off-board lanes read zeros at the bank quad their wrapped square would use
            base[m] = ok ? ((b * 64 + s2) * RS + h) * 16 : (ZB + ((s2 * RS) & 15) + h) * 16;
        }
#pragma unroll
        for (int cc = 0; cc < NCH; cc++) {
            const int ks = tap * NCH + cc;
            // next k-step's weight fragments: issued first so a whole k-step hides their latency
            const uint4 n0 = W[(size_t)(ks + 1) * CF * 64], n1 = W[(size_t)(ks + 1) * CF * 64 + 64];
            __builtin_amdgcn_sched_barrier(0);
            constexpr int LA = 3;                    // LDS reads kept in flight
            uint4 bq[LA];
#pragma unroll
            for (int m = 0; m < LA; m++) bq[m] = *reinterpret_cast<const uint4*>(ldsb + base[m] + cc * 64);
#pragma unroll
            for (int m = 0; m < MF; m++) {
                const uint4 bv = bq[m % LA];
                if (m + LA < MF) bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + base[m + LA] + cc * 64);
                if constexpr (sizeof(T) == 2) {
                    const bf16x8 A0 = __builtin_bit_cast(bf16x8, a0), A1 = __builtin_bit_cast(bf16x8, a1);
                    const bf16x8 Bv = __builtin_bit_cast(bf16x8, bv);
                    acc[m][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, Bv, acc[m][0], 0, 0, 0);
                    acc[m][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, Bv, acc[m][1], 0, 0, 0);
                } else {
                    const f32x4 A0 = __builtin_bit_cast(f32x4, a0), A1 = __builtin_bit_cast(f32x4, a1);
                    const f32x4 Bv = __builtin_bit_cast(f32x4, bv);
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        acc[m][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(A0[s], Bv[s], acc[m][0], 0, 0, 0);
                        acc[m][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[s], Bv[s], acc[m][1], 0, 0, 0);
                    }
                }
            }
            // pin the interleave: LA reads ahead, then [1 ds_read, the fragment's MFMAs] per fragment
            constexpr int MPM = sizeof(T) == 2 ? 2 : 8;
            __builtin_amdgcn_sched_group_barrier(0x100, LA, 0);
#pragma unroll
            for (int m = 0; m < MF; m++) {
                if (m + LA < MF) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, MPM, 0);
            }
            a0 = n0; a1 = n1;
            __builtin_amdgcn_sched_barrier(0);      // keep each k-step's reads with its MFMAs (no spills)
        }
    }

    // epilogue: bias (+ residual) + ReLU, 4 consecutive channels per lane
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int co = w * 32 + n * 16 + h * 4;
        const float4 bb = *reinterpret_cast<const float4*>(bias + co);
#pragma unroll
        for (int m = 0; m < MF; m++) {
            const int b = m >> 2;
            if (b >= nb) continue;
            const int sq = (m & 3) * 16 + (lane & 15);
            const size_t o = ((size_t)(row0 + b) * 64 + sq) * COUT + co;
            float v0 = acc[m][n][0] + bb.x, v1 = acc[m][n][1] + bb.y, v2 = acc[m][n][2] + bb.z,
                  v3 = acc[m][n][3] + bb.w;
            if constexpr (sizeof(T) == 2) {
                if constexpr (RESID) {
                    const bf16x4 r = *reinterpret_cast<const bf16x4*>(out + o);
                    v0 += (float)r[0]; v1 += (float)r[1]; v2 += (float)r[2]; v3 += (float)r[3];
                }
                bf16x4 y;
                y[0] = (__bf16)fmaxf(v0, 0.0f); y[1] = (__bf16)fmaxf(v1, 0.0f);
                y[2] = (__bf16)fmaxf(v2, 0.0f); y[3] = (__bf16)fmaxf(v3, 0.0f);
                *reinterpret_cast<bf16x4*>(out + o) = y;
            } else {
                if constexpr (RESID) {
                    const float4 r = *reinterpret_cast<const float4*>(out + o);
                    v0 += r.x; v1 += r.y; v2 += r.z; v3 += r.w;
                }
                *reinterpret_cast<float4*>(out + o) =
                    make_float4(fmaxf(v0, 0.0f), fmaxf(v1, 0.0f), fmaxf(v2, 0.0f), fmaxf(v3, 0.0f));
            }
        }
    }
}

// ------------------------------------------------------------------ heads
__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int F, typename T, bool SEARCH>
__global__ void __launch_bounds__(256)
heads_kernel(const T* __restrict__ x, const float* __restrict__ head, const int* __restrict__ count_ptr, int rows,
             float* __restrict__ pol_out, float* __restrict__ val_out, SearchOut so) {
    constexpr int XS = 64 * (F + 1) > 4096 ? 64 * (F + 1) : 4096;
    __shared__ float xs[XS];           // board activations, later the 4096 logits
    __shared__ float p1[32 * 64];
    __shared__ float v1[8 * 64];
    __shared__ float red[4 * 64];
    __shared__ float stat[8];
    const int count = count_ptr ? min(load_fresh(count_ptr), rows) : rows;
    const int row = vgpr_index(blockIdx.x);
    if (row >= count) return;
    const int tid = threadIdx.x;
    const HeadLayout L = HeadLayout::make(F);
    const T* xr = x + (size_t)row * 64 * F;
    for (int i = tid; i < 64 * F; i += 256) {
        const int sq = i / F, c = i - sq * F;
        xs[sq * (F + 1) + c] = to_f(xr[i]);
    }
    __syncthreads();
    const int sq = tid & 63;
    const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
    {   // 1x1 convs F -> 32 (policy) and F -> 8 (value), BN folded, ReLU
        float acc[10];
#pragma unroll
        for (int j = 0; j < 10; j++) acc[j] = 0.0f;
        const float* w40 = head + L.w40 + (size_t)g * 10 * F;
        for (int ci = 0; ci < F; ci++) {
            const float xv = xs[sq * (F + 1) + ci];
#pragma unroll
            for (int j = 0; j < 10; j++) acc[j] += w40[j * F + ci] * xv;
        }
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const int ch = g * 10 + j;
            const float v = fmaxf(acc[j] + head[L.b40 + ch], 0.0f);
            if (ch < 32) p1[ch * 64 + sq] = v; else v1[(ch - 32) * 64 + sq] = v;
        }
    }
    __syncthreads();
    float* lg = xs;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; j++) {   // 1x1 conv 32 -> 64: logits[c2*64 + sq]
        const int c2 = g * 16 + j;
        float l = 0.0f;
        for (int c1 = 0; c1 < 32; c1++) l += head[L.p2w + c2 * 32 + c1] * p1[c1 * 64 + sq];
        l += head[L.p2b + c2];
        lg[c2 * 64 + sq] = l;
        mx = fmaxf(mx, l);
    }
    // value hidden layer partials while logits settle
    {
        const int o = tid & 63, part = g;
        float a = 0.0f;
        for (int i = part * 128; i < part * 128 + 128; i++) a += v1[i] * head[L.l1w + i * 64 + o];
        red[part * 64 + o] = a;
    }
    mx = wave_max(mx);
    if ((tid & 63) == 0) stat[g] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(stat[0], stat[1]), fmaxf(stat[2], stat[3]));
    float s = 0.0f;
    for (int i = tid; i < 4096; i += 256) s += expf(lg[i] - mx);
    s = wave_sum(s);
    float hv = 0.0f;
    if (tid < 64) {
        const float hsum = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid] + head[L.l1b + tid];
        hv = fmaxf(hsum, 0.0f) * head[L.l2w + tid];
    }
    __syncthreads();
    if ((tid & 63) == 0) stat[4 + g] = s;
    if (tid < 64) {
        hv = wave_sum(hv);
        if (tid == 0) red[0] = tanhf(hv + head[L.l2b]);
    }
    __syncthreads();
    const float sum = stat[4] + stat[5] + stat[6] + stat[7];
    const float value = red[0];
    if constexpr (!SEARCH) {
        float* pr = pol_out + (size_t)row * 4096;
        for (int i = tid; i < 4096; i += 256) pr[i] = expf(lg[i] - mx) / sum;
        if (tid == 0) val_out[row] = value;
    } else {
        const int game = so.row_game[row], node = so.row_node[row];
        const Node nd = so.nodes[(size_t)game * so.NMAX + node];
        Edge* e = so.edges + (size_t)game * so.EMAX + nd.edge_begin;
        for (int i = tid; i < nd.nedges; i += 256) {
            const int idx = e[i].idx & azc::IDX_MASK;
            e[i].P = expf(lg[idx] - mx) / sum;
        }
        if (tid == 0) so.value[row] = value;
        if (so.log_cap > 0) {
            __shared__ int slot[2];
            if (tid == 0) {
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
            __syncthreads();
            if (slot[0] >= 0) {
                for (int i = tid; i < nd.nedges; i += 256) {
                    const int idx = e[i].idx & azc::IDX_MASK;
                    so.log_idx[slot[1] + i] = idx;
                    so.log_prior[slot[1] + i] = expf(lg[idx] - mx) / sum;
                }
            }
        }
    }
}

// ------------------------------------------------------------------ encoders
template <typename T>
__global__ void encode_rows_kernel(const azc::Pos* __restrict__ npos, int NMAX, const int* __restrict__ row_game,
                                   const int* __restrict__ row_node, const int* __restrict__ count_ptr, int rows,
                                   T* __restrict__ planes) {
    const int row = vgpr_index(blockIdx.x);
    const int count = count_ptr ? min(load_fresh(count_ptr), rows) : rows;
    if (row >= count) return;
    const int sq = threadIdx.x;
    const azc::Pos p = npos[(size_t)row_game[row] * NMAX + row_node[row]];
    T* o = planes + ((size_t)row * 64 + sq) * 32;
#pragma unroll
    for (int c = 0; c < 32; c++) o[c] = (T)(c < 19 ? azc::plane_value(p, c, sq) : 0.0f);
}

template <typename T>
__global__ void planes_from_nchw_kernel(const float* __restrict__ in, int rows, T* __restrict__ planes) {
    const int row = blockIdx.x, sq = threadIdx.x;
    if (row >= rows) return;
    T* o = planes + ((size_t)row * 64 + sq) * 32;
#pragma unroll
    for (int c = 0; c < 32; c++) o[c] = (T)(c < 19 ? in[((size_t)row * 19 + c) * 64 + sq] : 0.0f);
}

// synthetic evaluator -- the same definition the oracle uses
__global__ void synth_eval_kernel(const int* __restrict__ count_ptr, int rows, SearchOut so) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    const int count = count_ptr ? min(load_fresh(count_ptr), rows) : rows;
    if (row >= count) return;
    const int game = so.row_game[row], node = so.row_node[row];
    const Node nd = so.nodes[(size_t)game * so.NMAX + node];
    Edge* e = so.edges + (size_t)game * so.EMAX + nd.edge_begin;
    const uint64_t key = azc::fen_key(so.npos[(size_t)game * so.NMAX + node]);
    uint32_t total = 0;
    for (int i = 0; i < nd.nedges; i++) {
        const int idx = e[i].idx & azc::IDX_MASK;
        total += 1u + (uint32_t)(azc::splitmix64(key ^ ((uint64_t)(idx + 1) * 0x9E3779B97F4A7C15ULL)) >> 48);
    }
    int po = 0, r = -1;
    if (so.log_cap > 0) {
        r = atomicAdd(&so.ctr->log_count, 1);
        po = atomicAdd(&so.ctr->log_prior_count, (int)nd.nedges);
        if (r >= so.log_cap || po + nd.nedges > so.log_prior_cap) r = -1;
    }
    for (int i = 0; i < nd.nedges; i++) {
        const int idx = e[i].idx & azc::IDX_MASK;
        const uint32_t w = 1u + (uint32_t)(azc::splitmix64(key ^ ((uint64_t)(idx + 1) * 0x9E3779B97F4A7C15ULL)) >> 48);
        const float P = (float)w / (float)total;
        e[i].P = P;
        if (r >= 0) { so.log_idx[po + i] = idx; so.log_prior[po + i] = P; }
    }
    const int64_t v = (int64_t)(azc::splitmix64(key ^ 0x5BD1E9955BD1E995ULL) % 2001ULL) - 1000;
    const float value = (float)v / 1000.0f;
    so.value[row] = value;
    if (r >= 0) { so.log_key[r] = key; so.log_value[r] = value; so.log_off[r] = po; so.log_n[r] = nd.nedges; }
}

// ------------------------------------------------------------------ host side
namespace {

template <typename T>
int launch_conv(int F, int cin, bool resid, const void* in, void* out, const void* w, const float* b,
                const int* count, int rows, hipStream_t st) {
    constexpr bool BF = sizeof(T) == 2;
#define AZ_CONV(CI, CO, BP)                                                                                    \
    do {                                                                                                       \
        const int grid = (rows + BP - 1) / BP;                                                                 \
        if (resid)                                                                                             \
            conv3x3_kernel<CI, CO, BP, T, true><<<grid, CO * 2, 0, st>>>(                                      \
                (const T*)in, (T*)out, w, b, count, rows);                                                     \
        else                                                                                                   \
            conv3x3_kernel<CI, CO, BP, T, false><<<grid, CO * 2, 0, st>>>(                                     \
                (const T*)in, (T*)out, w, b, count, rows);                                                     \
        return hipGetLastError() == hipSuccess ? 0 : fail("conv launch failed");                               \
    } while (0)
    if (F == 32) { AZ_CONV(32, 32, 4); }
    if (F == 64) { if (cin == 32) AZ_CONV(32, 64, 4); AZ_CONV(64, 64, 4); }
    if (F == 128) { if (cin == 32) AZ_CONV(32, 128, 4); AZ_CONV(128, 128, 4); }
    if (F == 256) {
        if constexpr (BF) { if (cin == 32) AZ_CONV(32, 256, 4); AZ_CONV(256, 256, 4); }
        else { if (cin == 32) AZ_CONV(32, 256, 2); AZ_CONV(256, 256, 2); }
    }
#undef AZ_CONV
    return fail("unsupported filter count (32, 64, 128, 256)");
}

// fragment-swizzle one folded conv weight [cout][cin_real][9] for the MFMA A operand
std::vector<uint16_t> swizzle_bf16(const std::vector<float>& wf, int cout, int cin_real, int CIN) {
    const int nks = 9 * CIN / 32, CF = cout / 16;
    std::vector<uint16_t> o((size_t)(nks + 8) * CF * 64 * 8, 0);   // zero k-steps of prefetch padding
    for (int ks = 0; ks < nks; ks++)
        for (int cf = 0; cf < CF; cf++)
            for (int lane = 0; lane < 64; lane++)
                for (int j = 0; j < 8; j++) {
                    const int tap = ks / (CIN / 32);
                    const int ci = (ks % (CIN / 32)) * 32 + 8 * (lane >> 4) + j;
                    const int co = cf * 16 + (lane & 15);
                    const float v = ci < cin_real ? wf[((size_t)co * cin_real + ci) * 9 + tap] : 0.0f;
                    uint32_t u;
                    memcpy(&u, &v, 4);
                    u = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;   // round to nearest even
                    o[(((size_t)ks * CF + cf) * 64 + lane) * 8 + j] = (uint16_t)u;
                }
    return o;
}
std::vector<float> swizzle_f32(const std::vector<float>& wf, int cout, int cin_real, int CIN) {
    const int nkc = 9 * CIN / 16, CF = cout / 16;
    std::vector<float> o((size_t)(nkc + 8) * CF * 64 * 4, 0.0f);
    for (int kc = 0; kc < nkc; kc++)
        for (int cf = 0; cf < CF; cf++)
            for (int lane = 0; lane < 64; lane++)
                for (int s = 0; s < 4; s++) {
                    const int tap = kc / (CIN / 16);
                    const int ci = (kc % (CIN / 16)) * 16 + 4 * (lane >> 4) + s;
                    const int co = cf * 16 + (lane & 15);
                    o[(((size_t)kc * CF + cf) * 64 + lane) * 4 + s] =
                        ci < cin_real ? wf[((size_t)co * cin_real + ci) * 9 + tap] : 0.0f;
                }
    return o;
}

// The f32 input conv (19 planes) for the Winograd tower, packed: k-steps 0-8 = tap k, channels
// 0-15 (lane group h: channels 4h..4h+3, component = the MFMA k-slice); k-steps 9-11: slice s of
// k-step 9 + kl = tap 4 kl + s, lane group h = channel 16 + h (channel 19 and taps >= 9 zero);
// then 8 zero k-steps (ring refills past the end).  12 k-steps instead of the 18 of 32 padded
// channels (tower.hip conv32_in_packed)
std::vector<float> swizzle_f32_input_packed(const std::vector<float>& wf, int cout) {
    const int CF = cout / 16, NK = 12;
    std::vector<float> o((size_t)(NK + 8) * CF * 64 * 4, 0.0f);
    for (int k = 0; k < NK; k++)
        for (int cf = 0; cf < CF; cf++)
            for (int lane = 0; lane < 64; lane++)
                for (int s = 0; s < 4; s++) {
                    const int co = cf * 16 + (lane & 15), h = lane >> 4;
                    const int tap = k < 9 ? k : 4 * (k - 9) + s;
                    const int ci = k < 9 ? 4 * h + s : 16 + h;
                    o[(((size_t)k * CF + cf) * 64 + lane) * 4 + s] =
                        (tap < 9 && ci < 19) ? wf[((size_t)co * 19 + ci) * 9 + tap] : 0.0f;
                }
    return o;
}

// Winograd F(2x2,3x3) weights U = G g G^T (f64, rounded once), fragment-swizzled for the MFMA A
// operand: [ci/16][xi][co/16][lane][4], lane = co%16 + 16*((ci%16)/4), component ci%4, then 8 zero
// steps (ring refills past the end); tap = dy*3 + dx as in swizzle_f32
std::vector<float> winograd_f32(const std::vector<float>& wf, int F) {
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    const int CF = F / 16, NSTEP = (F / 16) * 16;
    std::vector<float> o((size_t)(NSTEP + 8) * CF * 64 * 4, 0.0f);
    for (int co = 0; co < F; co++)
        for (int ci = 0; ci < F; ci++) {
            const float* g = &wf[((size_t)co * F + ci) * 9];
            double gg[4][3];
            for (int a = 0; a < 4; a++)
                for (int j = 0; j < 3; j++) gg[a][j] = G[a][0] * g[0 * 3 + j] + G[a][1] * g[1 * 3 + j] + G[a][2] * g[2 * 3 + j];
            for (int a = 0; a < 4; a++)
                for (int b = 0; b < 4; b++) {
                    const double u = gg[a][0] * G[b][0] + gg[a][1] * G[b][1] + gg[a][2] * G[b][2];
                    const int step = (ci / 16) * 16 + a * 4 + b;
                    const int lane = (co % 16) + 16 * ((ci % 16) / 4);
                    o[(((size_t)step * CF + co / 16) * 64 + lane) * 4 + ci % 4] = (float)u;
                }
        }
    return o;
}

}  // namespace

int net_create(const az_net_desc* d, const float* wts, size_t n, int device, NetDev** out) {
    const int B = d->blocks, F = d->filters;
    if (!(F == 32 || F == 64 || F == 128 || F == 256)) return fail("filters must be 32, 64, 128 or 256");
    if (B < 0 || B > 64) return fail("blocks out of range");
    if (d->dtype != AZ_DTYPE_F32 && d->dtype != AZ_DTYPE_BF16) return fail("dtype must be AZ_DTYPE_F32/BF16");
    if (n != az_net_num_params(B, F)) return fail("weight count mismatch");
    AZ_HIP(hipSetDevice(device));
    NetDev* net = new NetDev();
    net->blocks = B; net->filters = F; net->dtype = d->dtype; net->device = device;
    if (const char* e = getenv("AZ_FUSED_TOWER")) net->fused = atoi(e) != 0;
    if (const char* e = getenv("AZ_WINOGRAD")) net->winograd = atoi(e) != 0;
    AZ_HIP(hipStreamCreateWithFlags(&net->stream, hipStreamNonBlocking));
    const float* p = wts;
    auto fold_conv = [&](int cin, const float* w, const float* bias, const float* bn) {
        const float *gamma = bn, *beta = bn + F, *mean = bn + 2 * F, *var = bn + 3 * F;
        std::vector<float> wf((size_t)F * cin * 9);
        std::vector<float> bf(F);
        for (int co = 0; co < F; co++) {
            const double sc = (double)gamma[co] / sqrt((double)var[co] + 1e-5);
            for (int k = 0; k < cin * 9; k++) wf[(size_t)co * cin * 9 + k] = (float)(w[(size_t)co * cin * 9 + k] * sc);
            bf[co] = (float)(((double)bias[co] - mean[co]) * sc + beta[co]);
        }
        const int CIN = cin == 19 ? 32 : cin;
        void* dw = nullptr;
        float* db = nullptr;
        size_t bytes = 0;
        if (d->dtype == AZ_DTYPE_BF16) {
            auto s = swizzle_bf16(wf, F, cin, CIN);
            bytes = s.size() * 2;
            if (hipMalloc(&dw, bytes) != hipSuccess) return -1;
            if (hipMemcpy(dw, s.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return -1;
        } else {
            auto s = swizzle_f32(wf, F, cin, CIN);
            bytes = s.size() * 4;
            if (hipMalloc(&dw, bytes) != hipSuccess) return -1;
            if (hipMemcpy(dw, s.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return -1;
        }
        net->conv_bytes.push_back(bytes);
        if (d->dtype == AZ_DTYPE_F32 && F >= 64 && cin == 19) {  // packed input conv for tower32w_kernel
            auto u = swizzle_f32_input_packed(wf, F);
            if (hipMalloc(&net->in_pk32, u.size() * 4) != hipSuccess) return -1;
            if (hipMemcpy(net->in_pk32, u.data(), u.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
            net->in_pk32_bytes = u.size() * 4;
        }
        if (d->dtype == AZ_DTYPE_F32 && F >= 64 && cin == F) {   // Winograd F(2x2,3x3) copy for tower32w_kernel
            auto u = winograd_f32(wf, F);
            void* du = nullptr;
            if (hipMalloc(&du, u.size() * 4) != hipSuccess) return -1;
            if (hipMemcpy(du, u.data(), u.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
            net->wino_w.push_back(du);
            net->wino_bytes.push_back(u.size() * 4);
        }
        if (hipMalloc(&db, F * 4) != hipSuccess) return -1;
        if (hipMemcpy(db, bf.data(), F * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
        net->conv_w.push_back(dw);
        net->conv_b.push_back(db);
        return 0;
    };
    // input conv + bn
    if (fold_conv(19, p, p + (size_t)F * 19 * 9, p + (size_t)F * 19 * 9 + F)) return fail("alloc conv");
    p += (size_t)F * 19 * 9 + F + 4 * F;
    for (int b = 0; b < B; b++) {
        for (int k = 0; k < 2; k++) {
            if (fold_conv(F, p, p + (size_t)F * F * 9, p + (size_t)F * F * 9 + F)) return fail("alloc conv");
            p += (size_t)F * F * 9 + F + 4 * F;
        }
    }
    // heads
    const HeadLayout L = HeadLayout::make(F);
    std::vector<float> hw(L.total, 0.0f);
    const float *p1w = p, *p1b = p1w + 32 * F, *pbn = p1b + 32, *p2w = pbn + 128, *p2b = p2w + 64 * 32;
    const float *vw = p2b + 64, *vb = vw + 8 * F, *vbn = vb + 8, *l1w = vbn + 32, *l1b = l1w + 512 * 64;
    const float *l2w = l1b + 64, *l2b = l2w + 64;
    auto fold1x1 = [&](int ch0, int cout, const float* w, const float* b, const float* bn) {
        for (int co = 0; co < cout; co++) {
            const double sc = (double)bn[co] / sqrt((double)bn[3 * cout + co] + 1e-5);
            for (int ci = 0; ci < F; ci++) hw[L.w40 + (size_t)(ch0 + co) * F + ci] = (float)(w[(size_t)co * F + ci] * sc);
            hw[L.b40 + ch0 + co] = (float)(((double)b[co] - bn[2 * cout + co]) * sc + bn[cout + co]);
        }
    };
    fold1x1(0, 32, p1w, p1b, pbn);
    fold1x1(32, 8, vw, vb, vbn);
    memcpy(&hw[L.p2w], p2w, 64 * 32 * 4);
    memcpy(&hw[L.p2b], p2b, 64 * 4);
    memcpy(&hw[L.l1w], l1w, 512 * 64 * 4);
    memcpy(&hw[L.l1b], l1b, 64 * 4);
    memcpy(&hw[L.l2w], l2w, 64 * 4);
    hw[L.l2b] = l2b[0];
    // policy 1x1 32->64 A-fragments: lane (l16, h) of tile cf holds rows cf*16 + l16, channels h + 4 ks
    for (int cf = 0; cf < 4; cf++)
        for (int lane = 0; lane < 64; lane++)
            for (int ks = 0; ks < 8; ks++)
                hw[L.p2f + ((size_t)cf * 64 + lane) * 8 + ks] = p2w[(cf * 16 + (lane & 15)) * 32 + (lane >> 4) + ks * 4];
    net->head_floats = L.total;
    AZ_HIP(hipMalloc(&net->head, L.total * 4));
    AZ_HIP(hipMemcpy(net->head, hw.data(), L.total * 4, hipMemcpyHostToDevice));
    {
        // the fused tower's heads run the 1x1 F->40 conv on bf16 MFMA with each f32 weight split
        // into hi = bf16(w) and lo = bf16(w - hi): [ks F/32][cf 3 (40 -> 48 rows)][hi, lo][lane][8],
        // lane = A-fragment row (co = cf*16 + lane%16) x k (ci = ks*32 + 8*(lane/16) + j)
        std::vector<uint16_t> fr((size_t)(F / 32) * 3 * 2 * 64 * 8, 0);
        auto bf = [](float v) {
            uint32_t u;
            memcpy(&u, &v, 4);
            return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
        };
        for (int ks = 0; ks < F / 32; ks++)
            for (int cf = 0; cf < 3; cf++)
                for (int lane = 0; lane < 64; lane++)
                    for (int j = 0; j < 8; j++) {
                        const int co = cf * 16 + (lane & 15), ci = ks * 32 + 8 * (lane >> 4) + j;
                        const float v = co < 40 ? hw[L.w40 + (size_t)co * F + ci] : 0.0f;
                        const uint16_t hi = bf(v);
                        const uint32_t hu = (uint32_t)hi << 16;
                        float hf;
                        memcpy(&hf, &hu, 4);
                        const size_t o = ((((size_t)ks * 3 + cf) * 2) * 64 + lane) * 8 + j;
                        fr[o] = hi;
                        fr[o + 64 * 8] = bf(v - hf);
                    }
        AZ_HIP(hipMalloc(&net->head_frag, fr.size() * 2));
        AZ_HIP(hipMemcpy(net->head_frag, fr.data(), fr.size() * 2, hipMemcpyHostToDevice));
        // f32 fused tower: the same 1x1 conv as exact f32 A-fragments of v_mfma_f32_16x16x4_f32,
        // [kc F/16][cf 3][lane][4]: co = cf*16 + lane%16, ci = kc*16 + 4*(lane/16) + s
        std::vector<float> f32fr((size_t)(F / 16) * 3 * 64 * 4, 0.0f);
        for (int kc = 0; kc < F / 16; kc++)
            for (int cf = 0; cf < 3; cf++)
                for (int lane = 0; lane < 64; lane++)
                    for (int s4 = 0; s4 < 4; s4++) {
                        const int co = cf * 16 + (lane & 15), ci = kc * 16 + 4 * (lane >> 4) + s4;
                        f32fr[(((size_t)kc * 3 + cf) * 64 + lane) * 4 + s4] = co < 40 ? hw[L.w40 + (size_t)co * F + ci] : 0.0f;
                    }
        AZ_HIP(hipMalloc(&net->head_frag32, f32fr.size() * 4));
        AZ_HIP(hipMemcpy(net->head_frag32, f32fr.data(), f32fr.size() * 4, hipMemcpyHostToDevice));
    }
    *out = net;
    return 0;
}

void net_destroy(NetDev* n) {
    if (!n) return;
    (void)hipSetDevice(n->device);
    for (void* w : n->conv_w) (void)hipFree(w);
    for (void* w : n->wino_w) (void)hipFree(w);
    for (float* b : n->conv_b) (void)hipFree(b);
    (void)hipFree(n->head);
    (void)hipFree(n->head_frag);
    (void)hipFree(n->head_frag32);
    (void)hipFree(n->in_pk32);
    (void)hipFree(n->x); (void)hipFree(n->h); (void)hipFree(n->planes);
    (void)hipFree(n->d_in); (void)hipFree(n->d_pol); (void)hipFree(n->d_val);
    if (n->stream) (void)hipStreamDestroy(n->stream);
    delete n;
}

int net_tower(NetDev* n, const void* planes, const int* count, int rows, void* x, void* h, hipStream_t st,
              hipEvent_t ev0, hipEvent_t ev1) {
    if (rows <= 0) return 0;
    const int F = n->filters;
    const bool bf = n->dtype == AZ_DTYPE_BF16;
    int rc = bf ? launch_conv<__bf16>(F, 32, false, planes, x, n->conv_w[0], n->conv_b[0], count, rows, st)
                : launch_conv<float>(F, 32, false, planes, x, n->conv_w[0], n->conv_b[0], count, rows, st);
    if (rc) return rc;
    for (int b = 0; b < n->blocks; b++) {
        const int i1 = 1 + 2 * b, i2 = 2 + 2 * b;
        if (b == 0 && ev0) (void)hipEventRecord(ev0, st);
        rc = bf ? launch_conv<__bf16>(F, F, false, x, h, n->conv_w[i1], n->conv_b[i1], count, rows, st)
                : launch_conv<float>(F, F, false, x, h, n->conv_w[i1], n->conv_b[i1], count, rows, st);
        if (rc) return rc;
        if (b == 0 && ev1) (void)hipEventRecord(ev1, st);
        rc = bf ? launch_conv<__bf16>(F, F, true, h, x, n->conv_w[i2], n->conv_b[i2], count, rows, st)
                : launch_conv<float>(F, F, true, h, x, n->conv_w[i2], n->conv_b[i2], count, rows, st);
        if (rc) return rc;
    }
    return 0;
}

template <bool SEARCH>
static int launch_heads(NetDev* n, const void* x, const int* count, int rows, float* pol, float* val,
                        const SearchOut& so, hipStream_t st) {
    const bool bf = n->dtype == AZ_DTYPE_BF16;
#define AZ_HEADS(FF)                                                                                       \
    if (n->filters == FF) {                                                                                \
        if (bf) heads_kernel<FF, __bf16, SEARCH><<<rows, 256, 0, st>>>((const __bf16*)x, n->head, count,  \
                                                                        rows, pol, val, so);               \
        else heads_kernel<FF, float, SEARCH><<<rows, 256, 0, st>>>((const float*)x, n->head, count, rows,  \
                                                                    pol, val, so);                         \
        return hipGetLastError() == hipSuccess ? 0 : fail("heads launch failed");                          \
    }
    AZ_HEADS(32) AZ_HEADS(64) AZ_HEADS(128) AZ_HEADS(256)
#undef AZ_HEADS
    return fail("unsupported filters");
}

int net_heads_dense(NetDev* n, const void* x, int rows, float* policy, float* value, hipStream_t st) {
    if (rows <= 0) return 0;
    SearchOut so;
    memset(&so, 0, sizeof(so));
    return launch_heads<false>(n, x, nullptr, rows, policy, value, so, st);
}

int net_heads_search(NetDev* n, const void* x, const int* count, int rows, const SearchOut& so, hipStream_t st) {
    if (rows <= 0) return 0;
    return launch_heads<true>(n, x, count, rows, nullptr, nullptr, so, st);
}

int net_encode_rows(NetDev* n, const azc::Pos* npos, int NMAX, const int* row_game, const int* row_node,
                    const int* count, int rows, void* planes, hipStream_t st) {
    if (rows <= 0) return 0;
    if (n->dtype == AZ_DTYPE_BF16)
        encode_rows_kernel<__bf16><<<rows, 64, 0, st>>>(npos, NMAX, row_game, row_node, count, rows, (__bf16*)planes);
    else
        encode_rows_kernel<float><<<rows, 64, 0, st>>>(npos, NMAX, row_game, row_node, count, rows, (float*)planes);
    return hipGetLastError() == hipSuccess ? 0 : fail("encode launch failed");
}

int net_planes_from_host_layout(NetDev* n, const float* d_in, int rows, void* planes, hipStream_t st) {
    if (rows <= 0) return 0;
    if (n->dtype == AZ_DTYPE_BF16)
        planes_from_nchw_kernel<__bf16><<<rows, 64, 0, st>>>(d_in, rows, (__bf16*)planes);
    else
        planes_from_nchw_kernel<float><<<rows, 64, 0, st>>>(d_in, rows, (float*)planes);
    return hipGetLastError() == hipSuccess ? 0 : fail("planes launch failed");
}

int synth_eval_rows(const int* count, int rows, const SearchOut& so, hipStream_t st) {
    if (rows <= 0) return 0;
    synth_eval_kernel<<<(rows + 63) / 64, 64, 0, st>>>(count, rows, so);
    return hipGetLastError() == hipSuccess ? 0 : fail("synth launch failed");
}

}  // namespace azi

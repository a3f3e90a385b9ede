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
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "az_internal.h"
#include "search_dev.h"
#include "wino.h"

// Tuning constants (the A/B logs under profiles/ measured each alternative):
//   TOWER_LA 4   bf16 tower: activation (B-fragment) LDS reads issued this many fragments ahead
//   TOWER_PF 2   bf16 tower: weight prefetch depth in k-steps (4 measured no faster)
//   HEADS_KPRE 64  value-FC rows per wave prefetched into registers before the heads' 1x1 conv
constexpr int TOWER_LA = 4, TOWER_PF = 2, HEADS_KPRE = 64;

namespace azi {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

struct TowerArgs {
    const uint4* w[1 + 2 * 40];    // swizzled conv weights (input conv, then conv1/conv2 per block)
    const float* b[1 + 2 * 40];    // folded biases
    const float* head;
    const uint4* head_frag;        // 1x1 F->40 head conv as bf16 hi/lo MFMA A-fragments (net.hip)
    const uint4* head_frag32;      // the same conv as f32 A-fragments (f32 tower)
    unsigned wbytes[1 + 2 * 40];   // allocation bytes of each w[i] (buffer-load range check)
    const uint4* ww[2 * 40];       // f32 Winograd weights of the residual convs (F = 256, tower32w_kernel)
    unsigned wwbytes[2 * 40];
    const uint4* w0pk;             // the input conv packed for tower32w_kernel (net.hip swizzle_f32_input_packed)
    unsigned w0pk_bytes;
    int blocks;
};

// BPB boards per workgroup; NCO 16-channel output fragments per wave; WB board groups.
// waves = (F / (16*NCO)) * WB
template <int F> struct TowerCfg;
// F = 256: 8 waves x 2 boards (16 waves, WB = 2, measured 10 % slower: spills); F = 64: 4 waves of 16
// channels, one per SIMD (NCO 2 left 2 SIMDs idle: C2 tower 52 -> 41 us), one board per workgroup
template <> struct TowerCfg<256> { static constexpr int BPB = 2, WB = 1, NCO = 2; };
template <> struct TowerCfg<128> { static constexpr int BPB = 4, WB = 1, NCO = 2; };
template <> struct TowerCfg<64> { static constexpr int BPB = 1, WB = 1, NCO = 1; };   // C2: 256 games -> 256 workgroups
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
template <int NCH> struct RingPF { static constexpr int PF = NCH >= TOWER_PF ? TOWER_PF : NCH; };

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
                                         int cw, int bw, int lane, unsigned wbytes, unsigned nbytes) {
    constexpr int NCH = CIN / 32;                     // 32-channel K chunks (4 slots)
    constexpr int CF = F / 16;
    constexpr int MF = BPW * 4;
    constexpr int KS = 9 * NCH;
    // weight fragments are prefetched PF k-steps ahead through a register ring; PF divides the
    // chunk count so the ring slot of every k-step is a compile-time constant
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
    // weight refills as buffer loads: SGPR descriptor + per-lane VGPR offset + the k-step's byte
    // offset in an SGPR -- no 64-bit VALU address adds (and their carry-hazard nops) in the MFMA
    // stream (C3 A/B: tower -2.7 %); num_records = the real allocation (this layer's k-steps + its
    // 8 zero k-steps of prefetch pad), past the last k-step the refills read the next layer
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)wsw, (short)0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rN = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(wnext ? wnext : wsw + (size_t)KS * CF * 64), (short)0,
        (int)(wnext ? nbytes : wbytes - (unsigned)KS * CF * 64 * 16), 0x00020000);
    const int voff = ((cw * NCO) * 64 + lane) * 16;
    // B-fragment (activation) reads run LA fragments ahead, across k-step and tap boundaries
    constexpr int LA = TOWER_LA < MF ? TOWER_LA : MF;
    static_assert(MF % LA == 0, "read-ahead ring must tile the fragment loop");
    // Per-tap LDS addresses of the B fragments, branch-free.  Valid taps read the shifted square;
    // off-board taps read the zero row at the same 16-B slot mod 16 (conflict-free): in_off and
    // zero_off are multiples of 256 B and every row offset keeps the slot, so the zero address is
    // zero_off | (valid-form address & 0xF0).
    const int lane_off = (((lane & 15) * RSI) + h) * 16;
    const int lr = (lane & 15) >> 3, lf = lane & 7;
    auto tap_bases = [&](int tap, int* base) {
        const int dr = tap / 3 - 1, df = tap % 3 - 1;
        const bool okf = (unsigned)(lf + df) < 8u;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bool ok = okf && (unsigned)(2 * q + lr + dr) < 8u;
#pragma unroll
            for (int bb = 0; bb < BPW; bb++) {
                const int m = bb * 4 + q;
                const int va = lane_off + (((bw * BPW + bb) * 64 + q * 16 + dr * 8 + df) * RSI) * 16 + in_off;
                const int vz = (va & 0xF0) | zero_off;
                base[m] = ok ? va : vz;
            }
        }
    };
    int bcur[MF], bnext[MF];
    uint4 bq[LA];
    tap_bases(0, bcur);
#pragma unroll
    for (int m = 0; m < LA; m++) bq[m] = *reinterpret_cast<const uint4*>(ldsb + bcur[m]);
    // the 9-tap loop fully unrolled: every tap's LDS offsets and off-board masks are compile-time
    // and no accumulator copies cross a loop edge (C3 A/B: tower -2.7 %)
#pragma unroll
    for (int tap = 0; tap < 9; tap++) {
        tap_bases(tap < 8 ? tap + 1 : 8, bnext);
#pragma unroll
        for (int c4 = 0; c4 < NCH; c4++) {
            uint4 a[NCO];
#pragma unroll
            for (int n = 0; n < NCO; n++) a[n] = wr[c4 % PF][n];
            // refill this ring slot with the k-step PF positions later in the sequence (the next
            // tap, or the next layer once past the end)
            {
                int kidx;
                bool nxt = false;
                if (c4 + PF < NCH) kidx = tap * NCH + c4 + PF;
                else if (tap < 8) kidx = (tap + 1) * NCH + c4 + PF - NCH;
                else { kidx = c4 + PF - NCH; nxt = true; }
                const int soff = kidx * CF * 64 * 16;
#pragma unroll
                for (int n = 0; n < NCO; n++)
                    wr[c4 % PF][n] = __builtin_bit_cast(
                        uint4, __builtin_amdgcn_raw_buffer_load_b128(nxt ? rN : rW, voff + n * 1024, soff, 0));
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < MF; m++) {
                const uint4 bv = bq[m % LA];
                if (m + LA < MF) {
                    bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bcur[m + LA] + c4 * 64);
                } else if (c4 + 1 < NCH) {                   // next k-step, same tap
                    bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bcur[m + LA - MF] + (c4 + 1) * 64);
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

// Heads v2 for NB boards [b0, b0 + NB) of the workgroup, from the LDS image x (bf16, or f32 when
// F32X, row stride RS slots), scratch in H; every one of the NT threads reaches every barrier.
//   A: 1x1 F->40 (policy conv 32 + value conv 8, BN folded) on v_mfma_f32_16x16x32_bf16 with the
//      f32 weights split into bf16 hi + lo fragments (16 mantissa bits; activations are bf16
//      already), or for f32 activations on v_mfma_f32_16x16x4_f32 (exact f32), bias + ReLU ->
//      p1v1 (f32);
//   B: policy 1x1 32->64 on v_mfma_f32_16x16x4_f32 (exact f32 products) -> 4096 logits;
//   C: value Linear 512->64 (K split over the waves), ReLU, Linear 64->1, tanh (f32 VALU);
//   then softmax over 4096 and the dense rows or, in search mode, the priors gathered at the
//   new node's legal edges (agent.rs:112-144, tree.rs:84-104).
template <int F> struct HeadsCfg { static constexpr int NB = F >= 128 ? 2 : 1; };
constexpr int HEADS_P1S = 80;                           // p1v1 row stride in floats (conflict-free B reads)
// NPART partial value-FC sums per (board, wave): 4 for the 4-wave f32 heads (WIDE)
constexpr int heads_npart(int NT, bool F32X) { return F32X && NT <= 256 ? 4 : 1; }
template <int NB, int NT, int NPART = 1> struct HeadsScratch {
    static constexpr int PV = 40 * HEADS_P1S, NW = NT / 64;
    static constexpr int P1 = 0, LG = P1 + NB * PV, RED = LG + NB * 4096, STAT = RED + NB * NW * 64 * NPART;
    static constexpr int FLOATS = STAT + NB * (2 * NW + 4);
};

template <int F, int RS, int NB, int NT, bool SEARCH, bool F32X = false>
__device__ __forceinline__ void heads_group(const char* __restrict__ xb, float* __restrict__ scr, int b0, int nb,
                                            int row0, int tid, const uint4* __restrict__ hfrag,
                                            const float* __restrict__ head, float* pol_out, float* val_out,
                                            const SearchOut& so, unsigned long long* tr = nullptr) {
    constexpr int NPART = heads_npart(NT, F32X);
    wino_stamp(tr, 1900);
    typedef HeadsScratch<NB, NT, NPART> S;
    constexpr int NW = S::NW, PV = S::PV, P1S = HEADS_P1S;
    const HeadLayout L = HeadLayout::make(F);
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 4, l16 = lane & 15;
    float* p1v1 = scr + S::P1;
    float* lg = scr + S::LG;
    float* red = scr + S::RED;
    float* stat = scr + S::STAT;                        // per board: [NW] max, [NW] sum, value, slot, prior off
    // weights of B and C are fetched into registers first: their latency hides behind A
    constexpr int TPW = 16 * NB / NW;                   // policy tiles per wave
    // value-FC rows prefetched per wave: all of them for the f32 towers' 4-wave workgroups (one wave
    // per SIMD, registers to spare)
    constexpr int KPMAX = (F32X && NW <= 4) ? 128 : HEADS_KPRE;
    constexpr int KP = 512 / NW, KPRE = KP < KPMAX ? KP : KPMAX;
    // 4-wave f32 heads: the value FC with each lane on 4 output units x every 4th row of the wave's
    // rows (16-byte coalesced weight reads, 4x fewer load instructions); partial sums per lane group
    constexpr bool WIDE = F32X && NW <= 4;
    // f32 with 4 waves: A's first KA 16-channel weight groups are requested before everything else,
    // so that the 1x1 conv does not wait behind the B / C prefetch
    constexpr int KA = (F32X && NW <= 4) ? (F / 16 < 4 ? F / 16 : 4) : 0;
    f32x4 hA[KA > 0 ? KA : 1][3];
    if constexpr (KA > 0) {
        if (w < 4 * NB) {
#pragma unroll
            for (int kc = 0; kc < KA; kc++)
#pragma unroll
                for (int cf = 0; cf < 3; cf++) hA[kc][cf] = __builtin_bit_cast(f32x4, hfrag[(kc * 3 + cf) * 64 + lane]);
        }
    }
    float pa[TPW > 0 ? TPW : 1][8];
#pragma unroll
    for (int k = 0; k < TPW; k++) {
        const int t = w + k * NW, cf = (t >> 2) & 3;
        if constexpr (KA > 0) {   // 4-wave f32 heads: the fragment copy, one 32-byte read per lane
            const f32x4* src = reinterpret_cast<const f32x4*>(head + L.p2f + ((size_t)cf * 64 + lane) * 8);
            const f32x4 lo = src[0], hi = src[1];
#pragma unroll
            for (int ks = 0; ks < 4; ks++) {
                pa[k][ks] = lo[ks];
                pa[k][ks + 4] = hi[ks];
            }
        } else {   // (the wider read costs the 8-wave F = 256 kernel a spill)
#pragma unroll
            for (int ks = 0; ks < 8; ks++) pa[k][ks] = head[L.p2w + (cf * 16 + l16) * 32 + h + ks * 4];
        }
    }
    float wv[KPRE > 0 && !WIDE ? KPRE : 1];
    f32x4 wq[WIDE ? KP / 4 : 1];
    if constexpr (WIDE) {
#pragma unroll
        for (int i = 0; i < KP / 4; i++)
#ifdef AZ_HEADS_NOVFC   // timing-only bound (wrong values): no value-FC weight stream
            wq[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#else
            wq[i] = *reinterpret_cast<const f32x4*>(head + L.l1w + (size_t)(w * KP + 4 * i + h) * 64 + 4 * l16);
#endif
    } else {
#pragma unroll
        for (int i = 0; i < KPRE; i++) wv[i] = head[L.l1w + (size_t)(w * KP + i) * 64 + lane];
    }
    // biases of A, B and the value head, and (search mode) the new node's record: requested here,
    // behind the weight prefetches, so that no phase ends on a dependent global load (C2 heads
    // stamps: ~1-2k cycles each)
    f32x4 b40v[3];
#pragma unroll
    for (int cf = 0; cf < 3; cf++) b40v[cf] = *reinterpret_cast<const f32x4*>(head + L.b40 + cf * 16 + 4 * h);
    f32x4 p2bv[TPW > 0 ? TPW : 1];
#pragma unroll
    for (int k = 0; k < TPW; k++)
        p2bv[k] = *reinterpret_cast<const f32x4*>(head + L.p2b + ((w + k * NW) >> 2 & 3) * 16 + 4 * h);
    const float l1bv = head[L.l1b + lane], l2wv = head[L.l2w + lane], l2bv = head[L.l2b];
    int sgame[NB], snode[NB];
    Node snd[NB];
    if constexpr (SEARCH) {
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            if (b0 + bb < nb) {
                const int row = vgpr_index(row0 + b0 + bb);
                sgame[bb] = so.row_game[row];
                snode[bb] = so.row_node[row];
                snd[bb] = so.nodes[(size_t)sgame[bb] * so.NMAX + snode[bb]];
            }
        }
    }
    // A
    for (int sfr = w; sfr < 4 * NB; sfr += NW) {
        const int bb = sfr >> 2, sq = (sfr & 3) * 16 + l16;
        const char* xr = xb + ((size_t)(b0 + bb) * 64 + sq) * RS * 16 + h * 16;
        f32x4 acc[3];
#pragma unroll
        for (int cf = 0; cf < 3; cf++) acc[cf] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (F32X) {
            // f32 activations: exact f32 products on v_mfma_f32_16x16x4_f32, one 16-channel k-chunk
            // (a float4 per lane) per 4 MFMAs
#pragma unroll
            for (int kc = 0; kc < KA; kc++) {
                const f32x4 Bv = *reinterpret_cast<const f32x4*>(xr + kc * 64);
#pragma unroll
                for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                    for (int cf = 0; cf < 3; cf++)
                        acc[cf] = __builtin_amdgcn_mfma_f32_16x16x4f32(hA[kc][cf][s4], Bv[s4], acc[cf], 0, 0, 0);
            }
#pragma unroll 4
            for (int kc = KA; kc < F / 16; kc++) {
                const f32x4 Bv = *reinterpret_cast<const f32x4*>(xr + kc * 64);
#pragma unroll
                for (int cf = 0; cf < 3; cf++) {
                    const f32x4 Av = __builtin_bit_cast(f32x4, hfrag[(kc * 3 + cf) * 64 + lane]);
#pragma unroll
                    for (int s4 = 0; s4 < 4; s4++)
                        acc[cf] = __builtin_amdgcn_mfma_f32_16x16x4f32(Av[s4], Bv[s4], acc[cf], 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < F / 32; ks++) {
                const bf16x8 Bv = *reinterpret_cast<const bf16x8*>(xr + ks * 64);
#pragma unroll
                for (int cf = 0; cf < 3; cf++)
#pragma unroll
                    for (int hl = 0; hl < 2; hl++)
                        acc[cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8, hfrag[((ks * 3 + cf) * 2 + hl) * 64 + lane]), Bv, acc[cf], 0, 0,
                            0);
            }
        }
#pragma unroll
        for (int cf = 0; cf < 3; cf++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int ch = cf * 16 + 4 * h + r;
                if (ch < 40) p1v1[bb * PV + ch * P1S + sq] = fmaxf(acc[cf][r] + b40v[cf][r], 0.0f);
            }
    }
    wino_stamp(tr, 1901);
    __syncthreads();
    wino_stamp(tr, 1902);
    // B
    float mxb[NB];
#pragma unroll
    for (int bb = 0; bb < NB; bb++) mxb[bb] = -INFINITY;
#pragma unroll
    for (int k = 0; k < TPW; k++) {
        const int t = w + k * NW;
        const int bb = t >> 4, cf = (t >> 2) & 3, sf = t & 3;
        const float* pb = p1v1 + bb * PV + h * P1S + sf * 16 + l16;
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < 8; ks++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[k][ks], pb[ks * 4 * P1S], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c2 = cf * 16 + 4 * h + r;
            const float l = acc[r] + p2bv[k][r];
            lg[bb * 4096 + c2 * 64 + sf * 16 + l16] = l;
#pragma unroll
            for (int q = 0; q < NB; q++)
                if (q == bb) mxb[q] = fmaxf(mxb[q], l);
        }
    }
    // C: value FC, wave w owns K rows [w*KP, (w+1)*KP), lane = output unit
    if constexpr (WIDE) {
        f32x4 a[NB];
#pragma unroll
        for (int bb = 0; bb < NB; bb++) a[bb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < KP / 4; i++) {
            const int k = w * KP + 4 * i + h, c = 32 + (k >> 6), sq = k & 63;
#pragma unroll
            for (int bb = 0; bb < NB; bb++) a[bb] += p1v1[bb * PV + c * P1S + sq] * wq[i];
        }
#pragma unroll
        for (int bb = 0; bb < NB; bb++) *reinterpret_cast<f32x4*>(red + ((bb * NW + w) * 4 + h) * 64 + 4 * l16) = a[bb];
    } else {
        float a[NB];
#pragma unroll
        for (int bb = 0; bb < NB; bb++) a[bb] = 0.0f;
#pragma unroll
        for (int i = 0; i < KP; i++) {
            const int k = w * KP + i, c = 32 + (k >> 6), sq = k & 63;
            const float wgt = i < KPRE ? wv[i < KPRE ? i : 0] : head[L.l1w + (size_t)k * 64 + lane];
#pragma unroll
            for (int bb = 0; bb < NB; bb++) a[bb] += p1v1[bb * PV + c * P1S + sq] * wgt;
        }
#pragma unroll
        for (int bb = 0; bb < NB; bb++) red[(bb * NW + w) * 64 + lane] = a[bb];
    }
#pragma unroll
    for (int bb = 0; bb < NB; bb++) {
        const float m = t_wave_max(mxb[bb]);
        if (lane == 0) stat[bb * (2 * NW + 4) + w] = m;
    }
    wino_stamp(tr, 1903);
    __syncthreads();
    wino_stamp(tr, 1904);
    float mx[NB];
#pragma unroll
    for (int bb = 0; bb < NB; bb++) {
        float m = -INFINITY;
        for (int i = 0; i < NW; i++) m = fmaxf(m, stat[bb * (2 * NW + 4) + i]);
        mx[bb] = m;
        float e = 0.0f;
        for (int i = tid; i < 4096; i += NT) e += expf(lg[bb * 4096 + i] - m);
        e = t_wave_sum(e);
        if (lane == 0) stat[bb * (2 * NW + 4) + NW + w] = e;
    }
    if (w < NB) {                                       // wave bb finishes board bb's value head
        const int bb = w;
        float hs = l1bv;
        for (int i = 0; i < NW * NPART; i++) hs += red[(bb * NW * NPART + i) * 64 + lane];
        float hv = t_wave_sum(fmaxf(hs, 0.0f) * l2wv);
        if (lane == 0) stat[bb * (2 * NW + 4) + 2 * NW] = tanhf(hv + l2bv);
    }
    if constexpr (SEARCH) {                             // thread 0 reserves eval-log slots
        if (tid == 0 && so.log_cap > 0) {
#pragma unroll
            for (int bb = 0; bb < NB; bb++) {
                int* sl = reinterpret_cast<int*>(stat + bb * (2 * NW + 4) + 2 * NW + 1);
                sl[0] = -1;
                if (b0 + bb >= nb) continue;
                const Node nd = snd[bb];
                const int r = atomicAdd(&so.ctr->log_count, 1);
                const int po = atomicAdd(&so.ctr->log_prior_count, (int)nd.nedges);
                sl[0] = (r < so.log_cap && po + nd.nedges <= so.log_prior_cap) ? r : -1;
                sl[1] = po;
            }
        }
    }
    wino_stamp(tr, 1905);
    __syncthreads();
    wino_stamp(tr, 1906);
#pragma unroll
    for (int bb = 0; bb < NB; bb++) {
        if (b0 + bb >= nb) break;
        const float* st = stat + bb * (2 * NW + 4);
        float sum = 0.0f;
        for (int i = 0; i < NW; i++) sum += st[NW + i];
        const float value = st[2 * NW];
        const int row = vgpr_index(row0 + b0 + bb);
        const float* lb = lg + bb * 4096;
        if constexpr (!SEARCH) {
            float* pr = pol_out + (size_t)row * 4096;
            for (int i = tid; i < 4096; i += NT) pr[i] = expf(lb[i] - mx[bb]) / sum;
            if (tid == 0) val_out[row] = value;
        } else {
            const int game = sgame[bb], node = snode[bb];
            const Node nd = snd[bb];
            Edge* e = so.edges + (size_t)game * so.EMAX + nd.edge_begin;
            const int* sl = reinterpret_cast<const int*>(st + 2 * NW + 1);
            const int slot = so.log_cap > 0 ? sl[0] : -1;
            for (int i = tid; i < nd.nedges; i += NT) {
                const int idx = e[i].idx & azc::IDX_MASK;
                const float P = expf(lb[idx] - mx[bb]) / sum;
                e[i].P = P;
                if (slot >= 0) {
                    so.log_idx[sl[1] + i] = idx;
                    so.log_prior[sl[1] + i] = P;
                }
            }
            if (tid == 0) {
                so.value[row] = value;
                if (slot >= 0) {
                    so.log_key[slot] = azc::fen_key(so.npos[(size_t)game * so.NMAX + node]);
                    so.log_value[slot] = value;
                    so.log_off[slot] = sl[1];
                    so.log_n[slot] = nd.nedges;
                }
            }
        }
    }
    __syncthreads();
}

// boards [row0, row0 + nb) through the bf16 tower, all waves of the workgroup
template <int F, bool SEARCH>
__device__ __forceinline__ void tower_board(const __bf16* __restrict__ planes, const TowerArgs& ta, int row0, int nb,
                                            float* __restrict__ pol_out, float* __restrict__ val_out,
                                            const SearchOut& so, int tid) {
    constexpr int BPB = TowerCfg<F>::BPB, WB = TowerCfg<F>::WB, BPW = BPB / WB, NCO = TowerCfg<F>::NCO;
    constexpr int NCW = F / (16 * NCO);
    constexpr int NT = NCW * WB * 64;
    constexpr int RSF = F / 8 + 2, RSI = 32 / 8 + 2;
    constexpr int XSZ = BPB * 64 * RSF;               // slots per activation buffer
    constexpr int ZN = 16 + F / 8;
    // h doubles as the heads' scratch: at least that large (small nets with 1 board per workgroup)
    constexpr int HSZ0 = (HeadsScratch<HeadsCfg<F>::NB, NT>::FLOATS * 4 + 15) / 16;
    constexpr int HSZ = ((XSZ > HSZ0 ? XSZ : HSZ0) + 15) / 16 * 16;
    __shared__ __attribute__((aligned(16))) uint4 lds[XSZ + HSZ + ZN];
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cw = w % NCW, bw = w / NCW;
    uint4* X = lds;
    uint4* H = lds + XSZ;
    const int zero_off = (XSZ + HSZ) * 16;
    const char* ldsb = reinterpret_cast<const char*>(lds);

    // stage the input planes [row][64][32] into H with row stride RSI
    if (planes) {
        const uint4* src = reinterpret_cast<const uint4*>(planes) + (size_t)row0 * 64 * 4;
        for (int c = tid; c < BPB * 64 * 4; c += NT) {
            const int rowi = c >> 2, slot = c & 3;
            H[rowi * RSI + slot] = rowi < nb * 64 ? src[c] : make_uint4(0, 0, 0, 0);
        }
    } else {
        // search mode without a planes buffer: to_tensor (chess.rs:191-245) straight from the
        // leaf's packed position into LDS, one thread per square -- the same per-element
        // conversion as encode_rows_kernel (net.hip), so the rows are bit-identical
        for (int rowi = tid; rowi < BPB * 64; rowi += NT) {
            uint4 q[4] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
            if (rowi < nb * 64) {
                const int row = vgpr_index(row0 + (rowi >> 6)), sq = rowi & 63;
                const azc::Pos p = so.npos[(size_t)so.row_game[row] * so.NMAX + so.row_node[row]];
                __bf16 v[32];
#pragma unroll
                for (int c = 0; c < 32; c++) v[c] = (__bf16)(c < 19 ? azc::plane_value(p, c, sq) : 0.0f);
                __builtin_memcpy(q, v, sizeof(v));
            }
#pragma unroll
            for (int k = 0; k < 4; k++) H[rowi * RSI + k] = q[k];
        }
    }
    for (int c = tid; c < ZN; c += NT) lds[XSZ + HSZ + c] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    {
        uint4 wr0[RingPF<1>::PF][NCO];
        ring_fill<1, F, NCO>(wr0, ta.w[0], cw, lane);
        conv_lds<32, RSI, F, RSF, BPW, NCO, false>(ldsb, X, XSZ * 16, zero_off, ta.w[0], nullptr, ta.b[0], wr0, cw,
                                                   bw, lane, ta.wbytes[0], 0u);
    }
    uint4 wr[RingPF<F / 32>::PF][NCO];
    if (ta.blocks > 0) ring_fill<F / 32, F, NCO>(wr, ta.w[1], cw, lane);
    for (int b = 0; b < ta.blocks; b++) {
        const uint4* after = b + 1 < ta.blocks ? ta.w[3 + 2 * b] : nullptr;
        const unsigned after_bytes = b + 1 < ta.blocks ? ta.wbytes[3 + 2 * b] : 0u;
        conv_lds<F, RSF, F, RSF, BPW, NCO, false>(ldsb, H, 0, zero_off, ta.w[1 + 2 * b], ta.w[2 + 2 * b],
                                                  ta.b[1 + 2 * b], wr, cw, bw, lane, ta.wbytes[1 + 2 * b],
                                                  ta.wbytes[2 + 2 * b]);
        conv_lds<F, RSF, F, RSF, BPW, NCO, true>(ldsb, X, XSZ * 16, zero_off, ta.w[2 + 2 * b], after,
                                                 ta.b[2 + 2 * b], wr, cw, bw, lane, ta.wbytes[2 + 2 * b], after_bytes);
    }
    // heads: NB boards at a time, scratch in H
    {
        constexpr int NB = HeadsCfg<F>::NB;
        static_assert(HeadsScratch<NB, NT>::FLOATS * 4 <= HSZ * 16, "heads scratch must fit in h");
        static_assert((16 * NB) % (NT / 64) == 0, "policy tiles must divide over the waves");
        for (int b0 = 0; b0 < BPB && b0 < nb; b0 += NB)
            heads_group<F, RSF, NB, NT, SEARCH>(ldsb, reinterpret_cast<float*>(H), b0, nb, row0, tid, ta.head_frag,
                                                ta.head, pol_out, val_out, so);
    }
}

template <int F, bool SEARCH>
__global__ void __launch_bounds__((F / (16 * TowerCfg<F>::NCO)) * TowerCfg<F>::WB * 64)
tower_kernel(const __bf16* __restrict__ planes, TowerArgs ta, const int* __restrict__ count_ptr, int rows,
             float* __restrict__ pol_out, float* __restrict__ val_out, SearchOut so) {
    constexpr int BPB = TowerCfg<F>::BPB;
    const int count = count_ptr ? min(load_fresh(count_ptr), rows) : rows;
    const int row0 = blockIdx.x * BPB;
    if (row0 >= count) return;
    tower_board<F, SEARCH>(planes, ta, row0, min(BPB, count - row0), pol_out, val_out, so, threadIdx.x);
}

// ====================================================================== f32 tower
// The reference evaluates in f32 (burn Cuda<f32>, main.rs:15,68; agent.rs:112-144).  This is the
// same fused structure at that precision: activations f32 in LDS, weights f32, every product
// an exact f32 FMA on v_mfma_f32_16x16x4_f32 (64 FLOP/clk/SIMD, the f32 peak, 157.3 TF).
// At 1/16 of the bf16 rate a k-step is long (NCO*MF*4 MFMAs x 32 cycles per wave), so operand
// delivery has ample slack: one board per workgroup (x and h f32 = 2 x 66 KB of LDS at F = 256),
// B fragments double-buffered one k-step ahead, weight fragments two k-steps ahead.
template <int F> struct Tower32Cfg;
template <> struct Tower32Cfg<256> { static constexpr int BPB = 1, WB = 1, NCO = 2; };   // 8 waves, 2 per SIMD
template <> struct Tower32Cfg<128> { static constexpr int BPB = 1, WB = 1, NCO = 2; };
template <> struct Tower32Cfg<64> { static constexpr int BPB = 1, WB = 1, NCO = 1; };
template <> struct Tower32Cfg<32> { static constexpr int BPB = 2, WB = 2, NCO = 1; };
constexpr int T32_PF = 2;  // weight k-steps in flight (register ring)

// One f32 3x3 conv layer LDS -> LDS.  IN: CIN channels (16-channel k-chunks = 4 float4 slots),
// row stride RSI slots; OUT: F channels, row stride RSO.  Wave (cw, bw) computes channels
// [16*NCO*cw, +16*NCO) of boards [bw*BPW, +BPW).  A = weights (16 co x 4 ci), B = activations
// (4 ci x 16 squares): one ds_read_b128 per lane holds 4 consecutive channels and feeds the 4
// MFMAs of a k-chunk (k = 4h + s).  wr: weight ring, holds this layer's first T32_PF k-steps on
// entry, the next layer's (rN) on exit.  The k-step byte offset rides in voffset, so the
// descriptor's num_records bounds every refill.
template <int CIN, int RSI, int F, int RSO, int BPW, int NCO, bool RESID>
__device__ __forceinline__ void conv32_lds(const char* __restrict__ ldsb, char* __restrict__ outb, int in_off,
                                           int zero_off, const __amdgpu_buffer_rsrc_t rW,
                                           const __amdgpu_buffer_rsrc_t rN, const float* __restrict__ bias,
                                           f32x4 (&wr)[T32_PF][NCO], int cw, int bw, int lane) {
    constexpr int NCH = CIN / 16;
    constexpr int CF = F / 16;
    constexpr int MF = BPW * 4;
    constexpr int PF = T32_PF;
    constexpr int KB = CF * 64 * 16;                  // bytes per k-step (all output fragments)
    static_assert(NCH % PF == 0, "ring slots must be compile-time");
    const int h = lane >> 4, l16 = lane & 15;
    f32x4 acc[MF][NCO];
#pragma unroll
    for (int n = 0; n < NCO; n++) {
        const float4 bn = *reinterpret_cast<const float4*>(bias + cw * 16 * NCO + n * 16 + h * 4);
#pragma unroll
        for (int m = 0; m < MF; m++) acc[m][n] = f32x4{bn.x, bn.y, bn.z, bn.w};
    }
    const int voff = ((cw * NCO) * 64 + lane) * 16;
    // per-tap B addresses, branch-free: off-board taps read the zero row at the same slot mod 16
    const int lane_off = ((l16 * RSI) + h) * 16;
    const int lr = l16 >> 3, lf = l16 & 7;
    auto tap_bases = [&](int tap, int* base) {
        const int dr = tap / 3 - 1, df = tap % 3 - 1;
        const bool okf = (unsigned)(lf + df) < 8u;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bool ok = okf && (unsigned)(2 * q + lr + dr) < 8u;
#pragma unroll
            for (int bb = 0; bb < BPW; bb++) {
                const int m = bb * 4 + q;
                const int va = lane_off + (((bw * BPW + bb) * 64 + q * 16 + dr * 8 + df) * RSI) * 16 + in_off;
                base[m] = ok ? va : ((va & 0xF0) | zero_off);
            }
        }
    };
    int bcur[MF], bnx[MF];
    f32x4 bq[MF], bn[MF];
    tap_bases(0, bcur);
#pragma unroll
    for (int m = 0; m < MF; m++) bq[m] = *reinterpret_cast<const f32x4*>(ldsb + bcur[m]);
#pragma unroll 1
    for (int tap = 0; tap < 9; tap++) {
        tap_bases(tap < 8 ? tap + 1 : 8, bnx);
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            // next k-step's B fragments (same tap, next chunk; or the next tap's first chunk) and the
            // weight refill are issued first: a whole k-step of MFMAs covers their latency
#pragma unroll
            for (int m = 0; m < MF; m++)
                bn[m] = *reinterpret_cast<const f32x4*>(ldsb + (c + 1 < NCH ? bcur[m] + (c + 1) * 64 : bnx[m]));
            f32x4 a[NCO];
#pragma unroll
            for (int n = 0; n < NCO; n++) a[n] = wr[c % PF][n];
            // refill the slot with the k-step PF later: this tap, the next tap, or the next layer
            {
                int kidx;
                bool nxt = false;
                if (c + PF < NCH) kidx = tap * NCH + c + PF;
                else if (tap < 8) kidx = (tap + 1) * NCH + c + PF - NCH;
                else { kidx = c + PF - NCH; nxt = true; }
#pragma unroll
                for (int n = 0; n < NCO; n++)
                    wr[c % PF][n] = __builtin_bit_cast(
                        f32x4, __builtin_amdgcn_raw_buffer_load_b128(nxt ? rN : rW, voff + n * 1024 + kidx * KB, 0, 0));
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int m = 0; m < MF; m++)
#pragma unroll
                    for (int n = 0; n < NCO; n++)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[n][s4], bq[m][s4], acc[m][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < MF; m++) bq[m] = bn[m];
        }
#pragma unroll
        for (int m = 0; m < MF; m++) bcur[m] = bnx[m];
    }
    // epilogue: (+ residual) + ReLU, 4 consecutive channels of one square per lane (16-B stores);
    // `in` and `out` are different buffers, the barrier after publishes `out`
#pragma unroll
    for (int n = 0; n < NCO; n++) {
        const int co = cw * 16 * NCO + n * 16 + h * 4;
        char* lane_base = outb + ((bw * BPW * 64 + l16) * RSO + (co >> 2)) * 16;
#pragma unroll
        for (int m = 0; m < MF; m++) {
            f32x4* dst = reinterpret_cast<f32x4*>(lane_base + ((m >> 2) * 64 + (m & 3) * 16) * RSO * 16);
            f32x4 v = acc[m][n];
            if constexpr (RESID) v += *dst;
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = fmaxf(v[r], 0.0f);
            *dst = v;
        }
    }
    __syncthreads();
}

// The f32 input conv of the Winograd tower (19 planes -> F, one board): the weights packed by
// net.hip swizzle_f32_input_packed -- k-steps 0-8: tap k, channels 0-15 (one ds_read_b128 of
// B per square fragment feeds 4 MFMAs, as conv32_lds); k-steps 9-11: MFMA slice s = tap 4 kl + s,
// lane group h = channel 16 + h (one ds_read_b32 per slice and square fragment).  12 k-steps of
// MFMAs instead of conv32_lds's 18 over 32 zero-padded channels.  Input planes at in_off (row
// stride RSI slots, channels 0-31), output F channels at outb (row stride RSO), + bias, ReLU.
// wr holds k-steps [0, T32_PF) on entry; rW covers the 12 k-steps and the 8 zero ones after.
template <int F, int RSI, int RSO, int NCO>
__device__ __forceinline__ void conv32_in_packed(const char* __restrict__ ldsb, char* __restrict__ outb, int in_off,
                                                 int zero_off, const __amdgpu_buffer_rsrc_t rW,
                                                 const float* __restrict__ bias, f32x4 (&wr)[T32_PF][NCO], int cw,
                                                 int lane) {
    constexpr int CF = F / 16, MF = 4, PF = T32_PF, KB = CF * 64 * 16, NK = 12;
    static_assert(NK % PF == 0, "ring slots must be compile-time");
    const int h = lane >> 4, l16 = lane & 15;
    f32x4 acc[MF][NCO];
#pragma unroll
    for (int n = 0; n < NCO; n++) {
        const float4 bn = *reinterpret_cast<const float4*>(bias + cw * 16 * NCO + n * 16 + h * 4);
#pragma unroll
        for (int m = 0; m < MF; m++) acc[m][n] = f32x4{bn.x, bn.y, bn.z, bn.w};
    }
    const int voff = ((cw * NCO) * 64 + lane) * 16;
    const int lr = l16 >> 3, lf = l16 & 7;
    // square fragment m, tap: the lane's square (2 m + lr, lf) shifted by the tap; off-board taps
    // read the zero row (channels 0-15: at the same slot mod 16, conflict-free as conv32_lds)
    auto tap_ok = [&](int tap, int m) {
        const int dr = tap / 3 - 1, df = tap % 3 - 1;
        return (unsigned)(lf + df) < 8u && (unsigned)(2 * m + lr + dr) < 8u;
    };
    auto row_addr = [&](int tap, int m) {   // byte offset of the shifted square's row
        const int dr = tap / 3 - 1, df = tap % 3 - 1;
        return ((l16 + m * 16 + dr * 8 + df) * RSI) * 16 + in_off;
    };
    auto main_addr = [&](int tap, int m) {
        const int va = row_addr(tap, m) + h * 16;
        return tap_ok(tap, m) ? va : ((va & 0xF0) | zero_off);
    };
    auto side_addr = [&](int tap, int m) {  // channel 16 + h
        return tap_ok(tap, m) ? row_addr(tap, m) + 64 + h * 4 : zero_off + 64 + h * 4;
    };
    f32x4 bq[MF];
#pragma unroll
    for (int m = 0; m < MF; m++) bq[m] = *reinterpret_cast<const f32x4*>(ldsb + main_addr(0, m));
#pragma unroll
    for (int k = 0; k < NK; k++) {
        // next k-step's B fragments first: a whole k-step of MFMAs covers their latency
        f32x4 bn[MF];
        if (k + 1 < 9) {
#pragma unroll
            for (int m = 0; m < MF; m++) bn[m] = *reinterpret_cast<const f32x4*>(ldsb + main_addr(k + 1, m));
        } else if (k + 1 < NK) {
            const int kl = k + 1 - 9;
#pragma unroll
            for (int m = 0; m < MF; m++)
#pragma unroll
                for (int s4 = 0; s4 < 4; s4++) {
                    const int tap = 4 * kl + s4;
                    bn[m][s4] = tap < 9 ? *reinterpret_cast<const float*>(ldsb + side_addr(tap, m)) : 0.0f;
                }
        }
        f32x4 a[NCO];
#pragma unroll
        for (int n = 0; n < NCO; n++) a[n] = wr[k % PF][n];
#pragma unroll
        for (int n = 0; n < NCO; n++)
            wr[k % PF][n] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rW, voff + n * 1024 + (k + PF) * KB, 0, 0));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
            for (int m = 0; m < MF; m++)
#pragma unroll
                for (int n = 0; n < NCO; n++)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[n][s4], bq[m][s4], acc[m][n], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (k + 1 < NK) {
#pragma unroll
            for (int m = 0; m < MF; m++) bq[m] = bn[m];
        }
    }
    // epilogue: + ReLU, 4 consecutive channels of one square per lane; the barrier after publishes it
#pragma unroll
    for (int n = 0; n < NCO; n++) {
        const int co = cw * 16 * NCO + n * 16 + h * 4;
        char* lane_base = outb + (l16 * RSO + (co >> 2)) * 16;
#pragma unroll
        for (int m = 0; m < MF; m++) {
            f32x4 v = acc[m][n];
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = fmaxf(v[r], 0.0f);
            *reinterpret_cast<f32x4*>(lane_base + (m * 16) * RSO * 16) = v;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t t32_rsrc(const uint4* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

// input planes [row][64][32] f32 -> H (row stride RSI slots): from a planes buffer, or in search
// mode to_tensor (chess.rs:191-245) from the leaf's packed position, one thread per square
template <int BPB, int RSI, int NT>
__device__ __forceinline__ void stage_planes_f32(uint4* H, const float* __restrict__ planes, const SearchOut& so,
                                                 int row0, int nb, int tid) {
    if (planes) {
        const uint4* src = reinterpret_cast<const uint4*>(planes) + (size_t)row0 * 64 * 8;
        for (int c = tid; c < BPB * 64 * 8; c += NT) {
            const int rowi = c >> 3, slot = c & 7;
            H[rowi * RSI + slot] = rowi < nb * 64 ? src[c] : make_uint4(0, 0, 0, 0);
        }
    } else {
        for (int rowi = tid; rowi < BPB * 64; rowi += NT) {
            float v[32];
#pragma unroll
            for (int c = 0; c < 32; c++) v[c] = 0.0f;
            if (rowi < nb * 64) {
                const int row = vgpr_index(row0 + (rowi >> 6)), sq = rowi & 63;
                const azc::Pos p = so.npos[(size_t)so.row_game[row] * so.NMAX + so.row_node[row]];
#pragma unroll
                for (int c = 0; c < 19; c++) v[c] = azc::plane_value(p, c, sq);
            }
            uint4 q[8];
            __builtin_memcpy(q, v, sizeof(v));
#pragma unroll
            for (int k = 0; k < 8; k++) H[rowi * RSI + k] = q[k];
        }
    }
}

template <int F, bool SEARCH>
__global__ void __launch_bounds__((F / (16 * Tower32Cfg<F>::NCO)) * Tower32Cfg<F>::WB * 64)
tower32_kernel(const float* __restrict__ planes, TowerArgs ta, const int* __restrict__ count_ptr, int rows,
               float* __restrict__ pol_out, float* __restrict__ val_out, SearchOut so) {
    constexpr int BPB = Tower32Cfg<F>::BPB, WB = Tower32Cfg<F>::WB, BPW = BPB / WB, NCO = Tower32Cfg<F>::NCO;
    constexpr int NCW = F / (16 * NCO);
    constexpr int NT = NCW * WB * 64;
    constexpr int RSF = F / 4 + 2, RSI = 32 / 4 + 2;  // f32 rows: F/4 slots + 2 pad (conflict-free b128 reads)
    constexpr int XSZ = BPB * 64 * RSF;
    constexpr int ZN = 16 + F / 4;
    constexpr int NBH = HeadsCfg<F>::NB < BPB ? HeadsCfg<F>::NB : BPB;
    constexpr int HSZ0 = (HeadsScratch<NBH, NT, heads_npart(NT, true)>::FLOATS * 4 + 15) / 16;
    constexpr int HSZ = ((XSZ > HSZ0 ? XSZ : HSZ0) + 15) / 16 * 16;
    static_assert(BPB * 64 * RSI <= HSZ, "input planes must fit in h");
    __shared__ __attribute__((aligned(16))) uint4 lds[XSZ + HSZ + ZN];
    const int count = count_ptr ? min(load_fresh(count_ptr), rows) : rows;
    const int row0 = blockIdx.x * BPB;
    if (row0 >= count) return;
    const int nb = min(BPB, count - row0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cw = w % NCW, bw = w / NCW;
    uint4* X = lds;
    uint4* H = lds + XSZ;
    const int zero_off = (XSZ + HSZ) * 16;
    const char* ldsb = reinterpret_cast<const char*>(lds);

    stage_planes_f32<BPB, RSI, NT>(H, planes, so, row0, nb, tid);
    for (int c = tid; c < ZN; c += NT) lds[XSZ + HSZ + c] = make_uint4(0, 0, 0, 0);
    __syncthreads();

    f32x4 wr[T32_PF][NCO];
    {
        const __amdgpu_buffer_rsrc_t r0 = t32_rsrc(ta.w[0], ta.wbytes[0]);
        const __amdgpu_buffer_rsrc_t r1 =
            ta.blocks > 0 ? t32_rsrc(ta.w[1], ta.wbytes[1]) : t32_rsrc(ta.w[0] + 18 * (F / 16) * 64, ta.wbytes[0] - 18 * (F / 16) * 1024);
        const int voff = ((cw * NCO) * 64 + lane) * 16;
#pragma unroll
        for (int i = 0; i < T32_PF; i++)
#pragma unroll
            for (int n = 0; n < NCO; n++)
                wr[i][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         r0, voff + n * 1024 + i * (F / 16) * 1024, 0, 0));
        conv32_lds<32, RSI, F, RSF, BPW, NCO, false>(ldsb, reinterpret_cast<char*>(X), XSZ * 16, zero_off, r0, r1,
                                                     ta.b[0], wr, cw, bw, lane);
    }
    for (int b = 0; b < ta.blocks; b++) {
        const int i1 = 1 + 2 * b, i2 = 2 + 2 * b;
        const __amdgpu_buffer_rsrc_t r1 = t32_rsrc(ta.w[i1], ta.wbytes[i1]);
        const __amdgpu_buffer_rsrc_t r2 = t32_rsrc(ta.w[i2], ta.wbytes[i2]);
        // after the block's second conv the ring prefetches the next block's first conv (or
        // reads this conv's zero pad after the last one)
        const __amdgpu_buffer_rsrc_t r3 =
            b + 1 < ta.blocks ? t32_rsrc(ta.w[i2 + 1], ta.wbytes[i2 + 1])
                              : t32_rsrc(ta.w[i2] + (size_t)9 * (F / 16) * (F / 16) * 64,
                                         ta.wbytes[i2] - 9u * (F / 16) * (F / 16) * 1024);
        conv32_lds<F, RSF, F, RSF, BPW, NCO, false>(ldsb, reinterpret_cast<char*>(H), 0, zero_off, r1, r2,
                                                    ta.b[i1], wr, cw, bw, lane);
        conv32_lds<F, RSF, F, RSF, BPW, NCO, true>(ldsb, reinterpret_cast<char*>(X), XSZ * 16, zero_off, r2, r3,
                                                   ta.b[i2], wr, cw, bw, lane);
    }
    static_assert(HeadsScratch<NBH, NT, heads_npart(NT, true)>::FLOATS * 4 <= HSZ * 16, "heads scratch must fit in h");
    static_assert((16 * NBH) % (NT / 64) == 0, "policy tiles must divide over the waves");
    for (int b0 = 0; b0 < BPB && b0 < nb; b0 += NBH)
        heads_group<F, RSF, NBH, NT, SEARCH, true>(ldsb, reinterpret_cast<float*>(H), b0, nb, row0, tid,
                                                   ta.head_frag32, ta.head, pol_out, val_out, so);
}


// ====================================================================== f32 Winograd tower
// The Winograd conv core is wino.h (shared with the training step).  conv_wino: one residual conv
// of the tower, LDS -> LDS: the core, then + residual (the block input x, kept in the registers of
// the wave that owns those outputs), ReLU, written back over the layer input in ACT.
#ifdef AZ_TOWER_TRACE
// trace build: per-wave phase stamps of the first AZ_TT_WG workgroups of the last launch
// (slot layout in tools/tower_trace.py); read back with az_tower_trace_read
constexpr int AZ_TT_WG = 8, AZ_TT_SLOTS = 2048;
__device__ unsigned long long az_tower_trace_buf[AZ_TT_WG * 8 * AZ_TT_SLOTS];
__device__ __forceinline__ unsigned long long* tt_slot(int w) {
    return blockIdx.x < AZ_TT_WG && w < 8 ? az_tower_trace_buf + (blockIdx.x * 8 + w) * AZ_TT_SLOTS : nullptr;
}
#else
__device__ __forceinline__ unsigned long long* tt_slot(int) { return nullptr; }
#endif

template <int F, bool RESID>
__device__ __forceinline__ void conv_wino(char* __restrict__ ldsb, int vbase,
                                          const __amdgpu_buffer_rsrc_t rW, const __amdgpu_buffer_rsrc_t rN,
                                          const float* __restrict__ bias,
                                          f32x4 (&wr)[WinoCfg<F>::PF][WinoCfg<F>::XS][WinoCfg<F>::NN],
                                          f32x4 (&xres)[WinoCfg<F>::NN][4], int w, int lane, bool pre_in,
                                          bool pre_out, int vsel, int* flag, int seq,
                                          unsigned long long* tr = nullptr) {
    constexpr int NN = WinoCfg<F>::NN, RS = F / 4 + 2, VBYTES = WinoCfg<F>::CH * 1024;
    const int l16 = lane & 15, h = lane >> 4;
    const int ty = l16 >> 2, tx = l16 & 3;
    const int co0 = w * 16 * NN + h * 4;
    auto out_addr = [&](int n, int a, int b) { return ((2 * ty + a) * 8 + 2 * tx + b) * RS * 16 + (co0 + n * 16) * 4; };
    // the residual: this wave's outputs of the block input, read before it is overwritten (keeping
    // them in registers from the previous conv's epilogue instead measured +0.4 % at C3)
    if constexpr (!RESID) {
#pragma unroll
        for (int n = 0; n < NN; n++)
#pragma unroll
            for (int q = 0; q < 4; q++) xres[n][q] = *reinterpret_cast<const f32x4*>(ldsb + out_addr(n, q >> 1, q & 1));
    }
    f32x4 y[NN][4];
    wino_stamp(tr, 0);
    // F = 64: the single chunk's V alternates between two buffers from conv to conv (vsel)
    wino_core<F>(ldsb, vbase + (F == 64 ? vsel * VBYTES : 0), rW, rN, bias, wr, w, lane, y, pre_in, tr);
    wino_stamp(tr, 10);
    f32x4 o[NN][4];
#pragma unroll
    for (int n = 0; n < NN; n++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            f32x4 v = y[n][q];
            if constexpr (RESID) v += xres[n][q];
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = fmaxf(v[r], 0.0f);
            *reinterpret_cast<f32x4*>(ldsb + out_addr(n, q >> 1, q & 1)) = v;
            o[n][q] = v;
        }
    wino_stamp(tr, 11);
    // F = 256: the next conv's chunk 0 is this conv's output channels 0-31, all written by wave 0;
    // the first wave of each SIMD pair finishes ahead of its partner, so waves 0-3
    // transform it into V[0] (free since the previous chunk barrier) while waves 4-7 finish, and the
    // next conv starts on its MFMAs after this barrier.  Wave 0's stores are published to waves 1-3
    // through an LDS flag (release / acquire at workgroup scope)
    if constexpr (F == 256) {
        if (pre_out && w < WinoCfg<F>::NWV / 2) {
            if (w == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            else
                while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != seq)
                    __builtin_amdgcn_s_sleep(1);
            WinoXf<F>(ldsb, vbase, w, lane).both(0, 0);
        }
    } else if constexpr (F == 64) {
        // F = 64: each wave's 16 output channels are a quarter of the next conv's single chunk;
        // the wave transforms them from its registers (DPP neighbour exchange) into the other V
        // buffer -- no ACT round trip, no barrier between the epilogue and the transform
        if (pre_out) wino_xform_regs<F>(o[0], ldsb + vbase + (1 - vsel) * VBYTES, w, lane);
        (void)flag; (void)seq;
    } else {
        (void)pre_out; (void)flag; (void)seq;
    }
    (void)o;
    __syncthreads();
}

// one board (batch row row0) through the Winograd f32 tower, all NWV waves of the workgroup
template <int F, bool SEARCH>
__device__ __forceinline__ void tower32w_board(const float* __restrict__ planes, const TowerArgs& ta, int row0,
                                                      float* __restrict__ pol_out, float* __restrict__ val_out,
                                                      const SearchOut& so, int tid) {
    constexpr int NWV = WinoCfg<F>::NWV, NT = NWV * 64, NN = WinoCfg<F>::NN, XS = WinoCfg<F>::XS;
    constexpr int RSF = F / 4 + 2, RSI = 32 / 4 + 2;
    constexpr int XSZ = 64 * RSF;                        // ACT, uint4 slots
    // both V buffers (one when a single chunk covers the input), also planes staging / heads scratch
    // (F = 64: two single-chunk buffers, alternating from conv to conv)
    constexpr int VSZ = (F / WinoCfg<F>::CH > 1 || F == 64 ? 2 : 1) * WinoCfg<F>::CH * 1024 / 16;
    constexpr int PF = WinoCfg<F>::PF;
    constexpr int ZN = 16 + F / 4;
    constexpr int PAD = WINO_PAD_SQ * RSF;               // zero squares either side of ACT
    static_assert(HeadsScratch<1, NT, heads_npart(NT, true)>::FLOATS * 4 <= VSZ * 16, "heads scratch must fit in V");
    static_assert(64 * RSI <= VSZ, "input planes must fit in V");
    __shared__ __attribute__((aligned(16))) uint4 lds[PAD + XSZ + PAD + VSZ + ZN + 1];
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint4* X = lds + PAD;
    uint4* V = X + XSZ + PAD;
    const int vbase = (XSZ + PAD) * 16;                  // offsets from ACT
    const int zero_off = (XSZ + PAD + VSZ) * 16;
    static_assert((XSZ + PAD + VSZ) * 16 % 256 == 0, "conv32_lds ORs the zero row's offset into the low byte");
    char* ldsb = reinterpret_cast<char*>(X);
    unsigned long long* tr = nullptr;
#ifdef AZ_TOWER_TRACE
    tr = tt_slot(w);
#endif
    wino_stamp(tr, 0);
    stage_planes_f32<1, RSI, NT>(V, planes, so, row0, 1, tid);
    for (int c = tid; c < ZN + 1; c += NT) V[VSZ + c] = make_uint4(0, 0, 0, 0);   // zero row + the pre-transform flag
    int* flag = reinterpret_cast<int*>(V + VSZ + ZN);
    for (int c = tid; c < PAD; c += NT) {
        lds[c] = make_uint4(0, 0, 0, 0);
        X[XSZ + c] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    wino_stamp(tr, 1);
    {   // input conv 19 -> F: direct, channels 16-18 of four taps packed per k-step (12 k-steps)
        f32x4 wr[T32_PF][NN];
        const __amdgpu_buffer_rsrc_t r0 = t32_rsrc(ta.w0pk, ta.w0pk_bytes);
        const int voff = ((w * NN) * 64 + lane) * 16;
#pragma unroll
        for (int i = 0; i < T32_PF; i++)
#pragma unroll
            for (int n = 0; n < NN; n++)
                wr[i][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         r0, voff + n * 1024 + i * (F / 16) * 1024, 0, 0));
        conv32_in_packed<F, RSI, RSF, NN>(ldsb, reinterpret_cast<char*>(X), vbase, zero_off, r0, ta.b[0], wr, w, lane);
    }
    wino_stamp(tr, 2);
    f32x4 xres[NN][4];
    f32x4 wring[PF][XS][NN];
    if (ta.blocks > 0) {
        const __amdgpu_buffer_rsrc_t r = t32_rsrc(ta.ww[0], ta.wwbytes[0]);
        const int voff = wino_voff<F>(w, lane);
#pragma unroll
        for (int i = 0; i < PF; i++)
#pragma unroll
            for (int xs = 0; xs < XS; xs++)
#pragma unroll
                for (int n = 0; n < NN; n++)
                    wring[i][xs][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                    r, voff + n * 1024 + wino_toff<F>(0, i * XS + xs), 0, 0));
    }
    for (int b = 0; b < ta.blocks; b++) {
        const unsigned wb3 = b + 1 < ta.blocks ? ta.wwbytes[2 * b + 2] : 0u;   // after the last conv: nothing (reads 0)
        const __amdgpu_buffer_rsrc_t r1 = t32_rsrc(ta.ww[2 * b], ta.wwbytes[2 * b]);
        const __amdgpu_buffer_rsrc_t r2 = t32_rsrc(ta.ww[2 * b + 1], ta.wwbytes[2 * b + 1]);
        const __amdgpu_buffer_rsrc_t r3 = t32_rsrc(b + 1 < ta.blocks ? ta.ww[2 * b + 2] : ta.ww[2 * b + 1], wb3);
        // F = 256 / 64: each conv transforms the next conv's chunk 0 at its end (conv_wino; C3 A/B
        // -0.3 % against the tail transform alone)
        constexpr bool PRE = F == 256 || F == 64;
        conv_wino<F, false>(ldsb, vbase, r1, r2, ta.b[1 + 2 * b], wring, xres, w, lane, PRE && b > 0, PRE, 0, flag,
                            2 * b + 1, tr ? tr + 3 + 64 * b : nullptr);
        conv_wino<F, true>(ldsb, vbase, r2, r3, ta.b[2 + 2 * b], wring, xres, w, lane, PRE, PRE && b + 1 < ta.blocks,
                           F == 64 ? 1 : 0, flag, 2 * b + 2, tr ? tr + 35 + 64 * b : nullptr);
    }
    heads_group<F, RSF, 1, NT, SEARCH, true>(ldsb, reinterpret_cast<float*>(V), 0, 1, row0, tid, ta.head_frag32, ta.head,
                                             pol_out, val_out, so, tr);
    wino_stamp(tr, 3 + 64 * 20);
}

template <int F, bool SEARCH>
__global__ void __launch_bounds__(WinoCfg<F>::NWV * 64)
tower32w_kernel(const float* __restrict__ planes, TowerArgs ta, const int* __restrict__ count_ptr, int rows,
                float* __restrict__ pol_out, float* __restrict__ val_out, SearchOut so) {
    const int count = count_ptr ? min(load_fresh(count_ptr), rows) : rows;
    if ((int)blockIdx.x >= count) return;
    tower32w_board<F, SEARCH>(planes, ta, blockIdx.x, pol_out, val_out, so, threadIdx.x);
}

// k_sims32w: simulation steps [step0, step1) of one game per workgroup, with no grid-wide step
// boundary.  A game's simulations only touch its own tree (tree.rs:180-207 runs them one after
// the other per game), so the workgroup of game g loops: wave 0 backs up the previous
// simulation, selects and expands (search_dev.h, the same functions as k_step); if the leaf
// needs the network, all waves evaluate it through the Winograd tower as batch row g, whose
// heads write the priors into the new node's edges and the value into value[g].  The last
// simulation is backed up before the kernel ends.  It replaces 2 launches per simulation step
// (k_step + the tower, each step waiting for the slowest game of both) when every game has a
// CU of its own (G <= CUs: C2), and is bit-identical to them (tests/test_gpu_search.py).
// Cross-wave hand-offs: the workgroup barriers carry workgroup-scope fences; every record written
// inside the kernel is read back through vector loads (vgpr_index), never the scalar cache.
// threads of the persistent kernel's workgroup: the Winograd f32 tower's, or the bf16 tower's
template <int F, bool BF16> struct SimsCfg { static constexpr int NT = WinoCfg<F>::NWV * 64; };
template <int F> struct SimsCfg<F, true> {
    static_assert(TowerCfg<F>::BPB == 1, "persistent bf16 kernel: one board per workgroup");
    static constexpr int NT = (F / (16 * TowerCfg<F>::NCO)) * TowerCfg<F>::WB * 64;
};
template <int F, bool BF16>
__global__ void __launch_bounds__((SimsCfg<F, BF16>::NT))
k_sims32w(Engine E, TowerArgs ta, SearchOut so, int step0, int step1) {
    __shared__ int s_kind;
    if (!E.active[vgpr_index(blockIdx.x)]) return;     // constant within a move
    for (int step = step0; step <= step1; step++) {
        // indices laundered per simulation so that neither phase's loop-invariant address
        // arithmetic is hoisted across the other (it would stay live through it and spill)
        const int tid = vgpr_index(threadIdx.x), g = vgpr_index(blockIdx.x);
        const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
        unsigned long long* tr = tt_slot(w);            // trace builds only (nullptr otherwise)
        wino_stamp(tr, 1910);
        if (w == 0) {
            if (step > step0) {                        // the previous simulation's backup
                backup_game(E, g, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
            wino_stamp(tr, 1911);
            int kind = X_NONE, nid = -1;
            if (step < step1) {
                select_game(E, g, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                wino_stamp(tr, 1912);
                kind = expand_leaf_wave<1>(E, g, lane, &nid, step);   // wave 0 only
                wino_stamp(tr, 1913);
                if (lane == 0) {
                    if (kind == X_ROW) {
                        E.row_game[g] = g;
                        E.row_node[g] = nid;
                        E.leaf_row[g] = g;
                        // per-game slot, summed at readout: two same-address atomics from every
                        // workgroup per simulation were waited on at the barrier below (batch_hist
                        // is read only for the timed steps, which never run in this kernel)
                        E.g_evals[g] += 1ull;   // g is in a VGPR: a vector load, never the scalar cache
                    } else if (kind == X_TERMINAL) {
                        atomicAdd(&E.ctr->terminal, 1ull);
                    } else if (kind == X_CACHED) {
                        atomicAdd(&E.ctr->cache_hits, 1ull);
                    }
                }
            }
            if (lane == 0) s_kind = kind;
        }
        __syncthreads();
        const int kind = s_kind;
        wino_stamp(tr, 1914);
        if (kind == X_ROW) {
            if constexpr (BF16) tower_board<F, true>(nullptr, ta, g, 1, nullptr, nullptr, so, tid);
            else tower32w_board<F, true>(nullptr, ta, g, nullptr, nullptr, so, tid);
        }
        __syncthreads();
        wino_stamp(tr, 1915);
    }
}

bool tower_supported(const NetDev* n) {
    return (n->dtype == AZ_DTYPE_BF16 || n->dtype == AZ_DTYPE_F32) && n->blocks <= 40 &&
           (n->filters == 256 || n->filters == 128 || n->filters == 64 || n->filters == 32);
}

bool wino_supported(const NetDev* n) {
    return n->dtype == AZ_DTYPE_F32 && n->winograd && n->filters >= 64 && (int)n->wino_w.size() == 2 * n->blocks &&
           n->in_pk32 != nullptr;
}

static TowerArgs tower_args(const NetDev* n) {
    TowerArgs ta;
    memset(&ta, 0, sizeof(ta));
    for (int i = 0; i < 1 + 2 * n->blocks; i++) {
        ta.w[i] = reinterpret_cast<const uint4*>(n->conv_w[i]);
        ta.b[i] = n->conv_b[i];
        ta.wbytes[i] = (unsigned)n->conv_bytes[i];
    }
    ta.head = n->head;
    ta.head_frag = reinterpret_cast<const uint4*>(n->head_frag);
    ta.head_frag32 = reinterpret_cast<const uint4*>(n->head_frag32);
    for (size_t i = 0; i < n->wino_w.size(); i++) {
        ta.ww[i] = reinterpret_cast<const uint4*>(n->wino_w[i]);
        ta.wwbytes[i] = (unsigned)n->wino_bytes[i];
    }
    ta.w0pk = reinterpret_cast<const uint4*>(n->in_pk32);
    ta.w0pk_bytes = (unsigned)n->in_pk32_bytes;
    ta.blocks = n->blocks;
    return ta;
}

bool sims_persistent_supported(const NetDev* n) {
    return tower_supported(n) && (wino_supported(n) || (n->dtype == AZ_DTYPE_BF16 && n->filters == 64));
}

// simulation steps [step0, step1) of every game through k_sims32w (one workgroup per game);
// ends with every simulation backed up
int sims_persistent(const NetDev* n, const Engine& E, const SearchOut& so, int step0, int step1, hipStream_t st) {
    if (step1 <= step0) return 0;
    if (!sims_persistent_supported(n)) return fail("persistent simulation kernel: needs the f32 Winograd tower or the bf16 64-filter tower");
    const TowerArgs ta = tower_args(n);
    if (n->dtype == AZ_DTYPE_BF16) {
        k_sims32w<64, true><<<E.G, SimsCfg<64, true>::NT, 0, st>>>(E, ta, so, step0, step1);
        return hipGetLastError() == hipSuccess ? 0 : fail("persistent simulation kernel launch failed");
    }
#define AZ_SIMS32W(FF)                                                                                  \
    if (n->filters == FF) {                                                                            \
        k_sims32w<FF, false><<<E.G, SimsCfg<FF, false>::NT, 0, st>>>(E, ta, so, step0, step1);          \
        return hipGetLastError() == hipSuccess ? 0 : fail("persistent simulation kernel launch failed"); \
    }
    AZ_SIMS32W(256) AZ_SIMS32W(128) AZ_SIMS32W(64)
#undef AZ_SIMS32W
    return fail("persistent simulation kernel: unsupported filters");
}

int tower_forward(NetDev* n, const void* planes, const int* count, int rows, float* pol, float* val,
                  const SearchOut* so, hipStream_t st) {
    if (rows <= 0) return 0;
    if (!tower_supported(n)) return fail("fused tower: unsupported net");
    if (!planes && (!so || !so->npos)) return fail("fused tower: no planes and no leaf positions to encode");
    TowerArgs ta = tower_args(n);
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
#define AZ_TOWER32(FF)                                                                                          \
    if (n->filters == FF) {                                                                                    \
        constexpr int BPB = Tower32Cfg<FF>::BPB;                                                               \
        constexpr int NT = (FF / (16 * Tower32Cfg<FF>::NCO)) * Tower32Cfg<FF>::WB * 64;                        \
        const int grid = (rows + BPB - 1) / BPB;                                                               \
        if (so) tower32_kernel<FF, true><<<grid, NT, 0, st>>>((const float*)planes, ta, count, rows, pol, val, s); \
        else tower32_kernel<FF, false><<<grid, NT, 0, st>>>((const float*)planes, ta, count, rows, pol, val, s);  \
        return hipGetLastError() == hipSuccess ? 0 : fail("f32 tower launch failed");                          \
    }
    if (n->dtype == AZ_DTYPE_F32) {
#define AZ_TOWER32W(FF)                                                                                       \
        if (n->filters == FF) {                                                                                \
            constexpr int NT = WinoCfg<FF>::NWV * 64;                                                          \
            if (so) tower32w_kernel<FF, true><<<rows, NT, 0, st>>>((const float*)planes, ta, count, rows, pol, val, s); \
            else tower32w_kernel<FF, false><<<rows, NT, 0, st>>>((const float*)planes, ta, count, rows, pol, val, s);  \
            return hipGetLastError() == hipSuccess ? 0 : fail("f32 Winograd tower launch failed");             \
        }
        if (wino_supported(n)) {
            AZ_TOWER32W(256) AZ_TOWER32W(128) AZ_TOWER32W(64)
        }
#undef AZ_TOWER32W
        AZ_TOWER32(256) AZ_TOWER32(128) AZ_TOWER32(64) AZ_TOWER32(32)
        return fail("fused tower: unsupported filters");
    }
    AZ_TOWER(256) AZ_TOWER(128) AZ_TOWER(64) AZ_TOWER(32)
#undef AZ_TOWER
#undef AZ_TOWER32
    return fail("fused tower: unsupported filters");
}

}  // namespace azi

#ifdef AZ_TOWER_TRACE
// trace build only: copy the phase stamps of the last tower launch (AZ_TT_WG x 8 waves x
// AZ_TT_SLOTS u64) to the host
extern "C" int az_tower_trace_read(unsigned long long* out, size_t n) {
    const size_t cap = sizeof(azi::az_tower_trace_buf) / sizeof(unsigned long long);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(azi::az_tower_trace_buf), (n < cap ? n : cap) * 8) == hipSuccess ? 0 : -1;
}
#endif

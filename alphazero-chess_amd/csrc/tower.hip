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

#ifndef AZ_TOWER_WB256
#define AZ_TOWER_WB256 1   // F=256: 8 waves x 2 boards (WB=2, 16 waves, measured 10% slower: spills)
#endif
#ifndef AZ_TOWER_NCO256
#define AZ_TOWER_NCO256 2
#endif
#ifndef AZ_TOWER_PRIO
#define AZ_TOWER_PRIO 0    // the two waves sharing a SIMD (w, w+4) take turns at issue priority, per
                           // PRIO k-steps: without it the older wave races ahead and the other
                           // finishes its layer alone, latency-bound (0 = off)
#endif
#ifndef AZ_TOWER_FLAGS
#define AZ_TOWER_FLAGS 0   // 1: F = 256 residual convs hand off through per-wave LDS flags (wait_done); measured 7 % slower
#endif
#ifndef AZ_TOWER_AACC
#define AZ_TOWER_AACC 0    // 1: residual-conv MFMAs as inline asm with AGPR accumulators
#endif
#ifndef AZ_TOWER_LA
#define AZ_TOWER_LA 4      // activation (B-fragment) LDS reads issued this many fragments ahead
#endif
#ifndef AZ_TOWER_ADAPT
#define AZ_TOWER_ADAPT 0   // N > 0: N times per tap, issue priority to whichever wave of a SIMD pair is behind
                           // (rolled tap loop: 1 = -1.0 % / -1.2 % tower time, 2 = +1.8 %, 4 = +3.9 %, 8 = +13 %;
                           // with the unrolled loop, 1 = +0.4 ... +1.5 %: off)
#endif
#ifndef AZ_TOWER_TAPU
#define AZ_TOWER_TAPU 9    // tap-loop unroll factor: 9 (full) = per-tap offsets and validity at compile time, no
                           // loop-carried register copies (C3 A/B: tower -2.7 %; 3 = neutral)
#endif
#ifndef AZ_TOWER_BUFW
#define AZ_TOWER_BUFW 1    // 1: weight refills as buffer loads (SGPR descriptor + k-step SGPR offset): C3 A/B tower -2.7 %
#endif
#ifndef AZ_TOWER_PAIRW
#define AZ_TOWER_PAIRW 0   // 1: explicit LDS wait per pair of activation fragments (fewer s_waitcnt in the MFMA stream)
#endif
#ifndef AZ_HEADS_KPRE
#define AZ_HEADS_KPRE 64   // value-FC rows per wave prefetched into registers before the 1x1 conv
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
    const uint4* head_frag;        // 1x1 F->40 head conv as bf16 hi/lo MFMA A-fragments (net.hip)
    const uint4* head_frag32;      // the same conv as f32 A-fragments (f32 tower)
    unsigned wbytes[1 + 2 * 40];   // allocation bytes of each w[i] (buffer-load range check)
    const uint4* ww[2 * 40];       // f32 Winograd weights of the residual convs (F = 256, tower32w_kernel)
    unsigned wwbytes[2 * 40];
    int blocks;
#if defined(AZ_TOWER_TRACE) || defined(AZ_WINO_TRACE)
    unsigned long long* trace;     // experiment only: [grid][TR_SLOTS] s_memrealtime stamps (100 MHz)
#endif
};
#if defined(AZ_TOWER_TRACE) || defined(AZ_WINO_TRACE)
constexpr int TR_SLOTS = 256;
#endif
#ifdef AZ_TOWER_TRACE
#define TR_STAMP(k)                                                                                  \
    do {                                                                                             \
        if (tid == 0) ta.trace[(size_t)blockIdx.x * TR_SLOTS + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define TR_STAMP(k) do { } while (0)
#endif

// BPB boards per workgroup; NCO 16-channel output fragments per wave; WB board groups.
// waves = (F / (16*NCO)) * WB
template <int F> struct TowerCfg;
template <> struct TowerCfg<256> { static constexpr int BPB = 2, WB = AZ_TOWER_WB256, NCO = AZ_TOWER_NCO256; };
template <> struct TowerCfg<128> { static constexpr int BPB = 4, WB = 1, NCO = 2; };
#ifndef AZ_TOWER_NCO64
#define AZ_TOWER_NCO64 1   // 4 waves of 16 channels: one per SIMD (NCO 2 = 2 waves left 2 SIMDs idle: C2 tower 52 -> 41 us)
#endif
template <> struct TowerCfg<64> { static constexpr int BPB = 1, WB = 1, NCO = AZ_TOWER_NCO64; };   // C2: 256 games -> 256 workgroups
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

// Layer hand-off without a workgroup barrier (NSPLIT = 2, F = 256): wave w publishes in
// done[w] the index of the last layer whose epilogue it has written; a wave reads input
// chunk c (32 channels, written by wave c) of layer L only once done[c] >= L - 1.  The k-steps
// run chunk group by chunk group (chunks 0-3, all taps; then 4-7), so the older waves 0-3,
// which win issue arbitration and finish a layer first, start the next one on their own
// chunks while their younger SIMD partners finish: no wave is left alone on its SIMD
// (measured: a lone wave keeps the matrix pipe ~40-50 % busy).  No WAR check is needed: a wave
// reaches its epilogue of layer L+1 only after reading every chunk of layer L, i.e. after every
// wave has finished layer L.  Bounded spin (a hand-off bug gives wrong results, not a hang).
__device__ __forceinline__ void wait_done(const int* done, int c0, int n, int need) {
    for (int c = c0; c < c0 + n; c++)
        for (int it = 0; *reinterpret_cast<const volatile int*>(done + c) < need && it < (1 << 20); it++)
            __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// wr: register ring holding this layer's next PF weight k-steps on entry; on exit it holds
// the first PF k-steps of `wnext` (the next layer with the same chunk count), or zeros.
template <int CIN, int RSI, int F, int RSO, int BPW, int NCO, bool RESID, int NSPLIT = 1>
__device__ __forceinline__ void conv_lds(const char* __restrict__ ldsb, uint4* __restrict__ out_lds, int in_off,
                                         int zero_off, const uint4* __restrict__ wsw, const uint4* __restrict__ wnext,
                                         const float* __restrict__ bias, uint4 (&wr)[RingPF<CIN / 32>::PF][NCO],
                                         int cw, int bw, int lane, int wpar, unsigned wbytes, unsigned nbytes,
                                         unsigned long long* trw = nullptr,
                                         int* done = nullptr, int lidx = 0, int* prog = nullptr, int wid = 0,
                                         int partner = -1) {
    constexpr int NCH = CIN / 32;                     // 32-channel K chunks (4 slots)
    if (trw && lane == 0) trw[0] = __builtin_amdgcn_s_memtime();
#ifdef AZ_TOWER_SOLO   // experiment only: waves 4-7 skip the residual convs (waves 0-3 run alone on their SIMDs)
    if (CIN > 32 && cw >= 4) {
        if (trw && lane == 0) trw[1] = trw[2] = __builtin_amdgcn_s_memtime();
        __syncthreads();
        if (trw && lane == 0) trw[3] = __builtin_amdgcn_s_memtime();
        return;
    }
#endif
    constexpr int CF = F / 16;
    constexpr int MF = BPW * 4;
    constexpr int KS = 9 * NCH;
    constexpr int CPH = NCH / NSPLIT;                 // chunks per group
    // weight fragments are prefetched PF k-steps ahead through a register ring; PF divides
    // the group's chunk count so the ring slot of every k-step is a compile-time constant
    constexpr int PF = RingPF<NCH>::PF;
    static_assert(NCH % NSPLIT == 0 && CPH % PF == 0, "prefetch depth must divide the chunk group");
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
    const uint4* Wn = wnext ? wnext + (size_t)(cw * NCO) * 64 + lane : W + (size_t)KS * CF * 64;
#if AZ_TOWER_BUFW
    // num_records = the real allocation (this layer's k-steps + its 8 zero k-steps of prefetch pad)
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)wsw, (short)0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rN = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(wnext ? wnext : wsw + (size_t)KS * CF * 64), (short)0,
        (int)(wnext ? nbytes : wbytes - (unsigned)KS * CF * 64 * 16), 0x00020000);
    const int voff = ((cw * NCO) * 64 + lane) * 16;
#endif
    // B-fragment (activation) reads run LA fragments ahead, across k-step and tap boundaries:
    // the first LA reads of step s+1 are issued inside step s (not across a chunk-group
    // boundary, where the producers' flags are checked first).
    constexpr int LA = AZ_TOWER_LA < MF ? AZ_TOWER_LA : MF;
    static_assert(MF % LA == 0, "read-ahead ring must tile the fragment loop");
    // Per-tap LDS addresses of the B fragments, branch-free (the tap loop is not unrolled, so
    // each tap boundary runs this once; a branchy form cost ~150 instructions per tap, which
    // a wave alone on its SIMD pays as matrix-pipe idle time).  Valid taps read the shifted
    // square; off-board taps read the zero row at the same 16-B slot mod 16 (conflict-free):
    // in_off and zero_off are multiples of 256 B and every row offset keeps the slot, so the
    // zero address is zero_off | (valid-form address & 0xF0).
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
#pragma unroll
    for (int half = 0; half < NSPLIT; half++) {
        if constexpr (NSPLIT > 1) wait_done(done, half * CPH, CPH, lidx - 1);
        tap_bases(0, bcur);
#pragma unroll
        for (int m = 0; m < LA; m++) bq[m] = *reinterpret_cast<const uint4*>(ldsb + bcur[m] + half * CPH * 64);
#if AZ_TOWER_ADAPT
        // progress-based issue priority between the two waves of a SIMD: the wave that is
        // behind its partner (by the partner's tap count read one tap earlier) issues first,
        // so both reach the layer barrier together instead of one finishing alone
        constexpr int ACH = AZ_TOWER_ADAPT < CPH ? AZ_TOWER_ADAPT : CPH;   // checks per tap
        constexpr bool ADAPT = F == 256 && CIN == F;  // two waves per SIMD (C2's 4-wave tower: +5 % without this guard)
        int other = lidx * 9 * ACH;
#endif
#pragma unroll AZ_TOWER_TAPU
        for (int tap = 0; tap < 9; tap++) {
            tap_bases(tap < 8 ? tap + 1 : 8, bnext);
#pragma unroll
            for (int c4 = 0; c4 < CPH; c4++) {
                const int cc = half * CPH + c4;
#if AZ_TOWER_ADAPT
                if (ADAPT && partner >= 0 && c4 % (CPH / ACH) == 0) {
                    const int mine = (lidx * 9 + tap) * ACH + c4 / (CPH / ACH);
                    // LDS-typed accesses: through the generic pointer they compile to flat ops,
                    // which count against vmcnt too and stall the weight-prefetch waits
                    typedef __attribute__((address_space(3))) volatile int lds_vint;
                    if (lane == 0) *(lds_vint*)(prog + wid) = mine;
                    if (mine > other) __builtin_amdgcn_s_setprio(0);
                    else __builtin_amdgcn_s_setprio(1);
                    other = __builtin_amdgcn_readfirstlane(*(lds_vint*)(prog + partner));
                }
#endif
                if constexpr (AZ_TOWER_PRIO > 0) {
                    if ((((cc / AZ_TOWER_PRIO) & 1) ^ wpar) != 0) __builtin_amdgcn_s_setprio(1);
                    else __builtin_amdgcn_s_setprio(0);
                }
                uint4 a[NCO];
#pragma unroll
                for (int n = 0; n < NCO; n++) a[n] = wr[c4 % PF][n];
                // refill this ring slot with the k-step PF positions later in the sequence
                // (the next tap, the next chunk group, or the next layer once past the end)
                const uint4* Wsrc;
                if (c4 + PF < CPH) Wsrc = W + (size_t)(tap * NCH + cc + PF) * CF * 64;
                else if (tap < 8) Wsrc = W + (size_t)((tap + 1) * NCH + half * CPH + c4 + PF - CPH) * CF * 64;
                else if (half + 1 < NSPLIT) Wsrc = W + (size_t)((half + 1) * CPH + c4 + PF - CPH) * CF * 64;
                else Wsrc = Wn + (size_t)(c4 + PF - CPH) * CF * 64;
#if AZ_TOWER_BUFW
                // buffer loads: SGPR descriptor + per-lane VGPR offset + the k-step's byte offset in an
                // SGPR -- no 64-bit VALU address adds (and their carry-hazard nops) in the MFMA stream
                {
                    int kidx;
                    bool nxt = false;
                    if (c4 + PF < CPH) kidx = tap * NCH + cc + PF;
                    else if (tap < 8) kidx = (tap + 1) * NCH + half * CPH + c4 + PF - CPH;
                    else if (half + 1 < NSPLIT) kidx = (half + 1) * CPH + c4 + PF - CPH;
                    else { kidx = c4 + PF - CPH; nxt = true; }
                    const int soff = kidx * CF * 64 * 16;
#pragma unroll
                    for (int n = 0; n < NCO; n++)
                        wr[c4 % PF][n] = __builtin_bit_cast(
                            uint4, __builtin_amdgcn_raw_buffer_load_b128(nxt ? rN : rW, voff + n * 1024, soff, 0));
                    (void)Wsrc;
                }
#else
#pragma unroll
#if defined(AZ_TOWER_L1W)   // experiment only: every k-step re-reads k-steps 0..1 (L1-resident weights)
                for (int n = 0; n < NCO; n++) wr[c4 % PF][n] = W[(size_t)((c4 + PF) & 1) * CF * 64 + n * 64];
                (void)Wsrc;
#else
                for (int n = 0; n < NCO; n++) wr[c4 % PF][n] = Wsrc[n * 64];
#endif
#endif
                __builtin_amdgcn_sched_barrier(0);
                const bool last_of_group = tap == 8 && c4 + 1 == CPH && half + 1 < NSPLIT;
#pragma unroll
                for (int m = 0; m < MF; m++) {
#if AZ_TOWER_PAIRW
                    // one LDS wait per fragment pair (fragments m, m+1 done: LA-2 reads left in
                    // flight); the compiler's own per-fragment waits become redundant and drop
                    if ((m & 1) == 0) __builtin_amdgcn_s_waitcnt(0xC07F & ~0x0F00 | ((LA - 2) << 8));
#endif
                    const uint4 bv = bq[m % LA];
#ifndef AZ_TOWER_NOLDSR   // (experiment only: no activation reads inside the loop)
                    if (m + LA < MF) {
                        bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bcur[m + LA] + cc * 64);
                    } else if (c4 + 1 < CPH) {                   // next k-step, same tap
                        bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bcur[m + LA - MF] + (cc + 1) * 64);
                    } else if (!last_of_group) {                 // first k-step of the next tap
                        bq[m % LA] = *reinterpret_cast<const uint4*>(ldsb + bnext[m + LA - MF] + half * CPH * 64);
                    }
#endif
                    const bf16x8 Bv = __builtin_bit_cast(bf16x8, bv);
#pragma unroll
                    for (int n = 0; n < NCO; n++) {
#if AZ_TOWER_AACC
                        // accumulators pinned to AGPRs: no VGPR renaming of C/D through the B registers
                        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                                     : "+a"(acc[m][n])
                                     : "v"(__builtin_bit_cast(bf16x8, a[n])), "v"(Bv));
#else
                        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[n]), Bv,
                                                                            acc[m][n], 0, 0, 0);
#endif
                    }
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
    }
    (void)KS;
#if AZ_TOWER_AACC
    // the compiler does not see the asm MFMAs: cover the XDL-write -> VALU-read hazard by hand
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#endif
    if constexpr (AZ_TOWER_PRIO > 0 || (AZ_TOWER_ADAPT && F == 256 && CIN == F)) __builtin_amdgcn_s_setprio(0);
    if (trw && lane == 0) trw[1] = __builtin_amdgcn_s_memtime();
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
    if (trw && lane == 0) trw[2] = __builtin_amdgcn_s_memtime();
    if constexpr (NSPLIT > 1) {
        // publish: this wave's LDS writes complete, then done[cw] = lidx
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) *reinterpret_cast<volatile int*>(done + cw) = lidx;
    } else {
        __syncthreads();
    }
    if (trw && lane == 0) trw[3] = __builtin_amdgcn_s_memtime();
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
                                            const SearchOut& so, unsigned long long* trh = nullptr) {
    constexpr int NPART = heads_npart(NT, F32X);
    typedef HeadsScratch<NB, NT, NPART> S;
    constexpr int NW = S::NW, PV = S::PV, P1S = HEADS_P1S;
    const HeadLayout L = HeadLayout::make(F);
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 4, l16 = lane & 15;
    float* p1v1 = scr + S::P1;
    float* lg = scr + S::LG;
    float* red = scr + S::RED;
    float* stat = scr + S::STAT;                        // per board: [NW] max, [NW] sum, value, slot, prior off
#define HT_STAMP(k) do { if (F32X && trh && tid == 0) trh[k] = __builtin_amdgcn_s_memtime(); } while (0)   // f32 towers only
    HT_STAMP(3);
    // weights of B and C are fetched into registers first: their latency hides behind A
    constexpr int TPW = 16 * NB / NW;                   // policy tiles per wave
    // value-FC rows prefetched per wave: all of them for the f32 towers' 4-wave workgroups (one wave
    // per SIMD, registers to spare)
    constexpr int KPMAX = (F32X && NW <= 4) ? 128 : AZ_HEADS_KPRE;
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
            wq[i] = *reinterpret_cast<const f32x4*>(head + L.l1w + (size_t)(w * KP + 4 * i + h) * 64 + 4 * l16);
    } else {
#pragma unroll
        for (int i = 0; i < KPRE; i++) wv[i] = head[L.l1w + (size_t)(w * KP + i) * 64 + lane];
    }
    HT_STAMP(4);
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
        HT_STAMP(5);
#pragma unroll
        for (int cf = 0; cf < 3; cf++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int ch = cf * 16 + 4 * h + r;
                if (ch < 40) p1v1[bb * PV + ch * P1S + sq] = fmaxf(acc[cf][r] + head[L.b40 + ch], 0.0f);
            }
    }
    __syncthreads();
    if (trh && tid == 0) trh[0] = F32X ? __builtin_amdgcn_s_memtime() : __builtin_amdgcn_s_memrealtime();
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
            const float l = acc[r] + head[L.p2b + c2];
            lg[bb * 4096 + c2 * 64 + sf * 16 + l16] = l;
#pragma unroll
            for (int q = 0; q < NB; q++)
                if (q == bb) mxb[q] = fmaxf(mxb[q], l);
        }
    }
    HT_STAMP(16);
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
    HT_STAMP(17);
#pragma unroll
    for (int bb = 0; bb < NB; bb++) {
        const float m = t_wave_max(mxb[bb]);
        if (lane == 0) stat[bb * (2 * NW + 4) + w] = m;
    }
    __syncthreads();
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
        float hs = head[L.l1b + lane];
        for (int i = 0; i < NW * NPART; i++) hs += red[(bb * NW * NPART + i) * 64 + lane];
        float hv = t_wave_sum(fmaxf(hs, 0.0f) * head[L.l2w + lane]);
        if (lane == 0) stat[bb * (2 * NW + 4) + 2 * NW] = tanhf(hv + head[L.l2b]);
    }
    if (trh && tid == 0) trh[1] = F32X ? __builtin_amdgcn_s_memtime() : __builtin_amdgcn_s_memrealtime();
    if constexpr (SEARCH) {                             // thread 0 reserves eval-log slots
        if (tid == 0 && so.log_cap > 0) {
#pragma unroll
            for (int bb = 0; bb < NB; bb++) {
                int* sl = reinterpret_cast<int*>(stat + bb * (2 * NW + 4) + 2 * NW + 1);
                sl[0] = -1;
                if (b0 + bb >= nb) continue;
                const int row = vgpr_index(row0 + b0 + bb);
                const int game = so.row_game[row], node = so.row_node[row];
                const Node nd = so.nodes[(size_t)game * so.NMAX + node];
                const int r = atomicAdd(&so.ctr->log_count, 1);
                const int po = atomicAdd(&so.ctr->log_prior_count, (int)nd.nedges);
                sl[0] = (r < so.log_cap && po + nd.nedges <= so.log_prior_cap) ? r : -1;
                sl[1] = po;
            }
        }
    }
    __syncthreads();
    if (trh && tid == 0) trh[2] = F32X ? __builtin_amdgcn_s_memtime() : __builtin_amdgcn_s_memrealtime();
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
            const int game = so.row_game[row], node = so.row_node[row];
            const Node nd = so.nodes[(size_t)game * so.NMAX + node];
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
#undef HT_STAMP

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
    // chunk-group split + per-wave done flags (no barrier between residual convs): F = 256 only
    constexpr int NSP = (AZ_TOWER_FLAGS && F == 256 && WB == 1) ? 2 : 1;
    __shared__ __attribute__((aligned(16))) uint4 lds[XSZ + HSZ + ZN + 6];
    const int lane = tid & 63;
    TR_STAMP(0);
#ifdef AZ_TOWER_TRACE
    if (tid == 0) ta.trace[(size_t)blockIdx.x * TR_SLOTS + 112] = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        unsigned hww;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hww));
        ta.trace[(size_t)blockIdx.x * TR_SLOTS + 114 + (tid >> 6)] = hww;
    }
    if (tid == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        ta.trace[(size_t)blockIdx.x * TR_SLOTS + 47] = ((unsigned long long)xcc << 32) | hw;
    }
#endif
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cw = w % NCW, bw = w / NCW;
    const int wpar = (w >> 2) & 1;                    // waves w and w+4 share a SIMD
#ifdef AZ_TOWER_YPRIO   // experiment: static priority for the younger half (guide T5 static form)
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
#endif
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
    int* done = reinterpret_cast<int*>(lds + XSZ + HSZ + ZN);   // [8] last layer whose epilogue wave w wrote
    if (tid < 8) done[tid] = 0;                              // layer 0 = the input conv (barrier after it)
    int* prog = done + 8;                                    // [8] tap counter per wave, [8] its SIMD
#if AZ_TOWER_ADAPT
    if constexpr (F == 256) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        if (lane == 0) { prog[8 + (tid >> 6)] = (hw >> 4) & 3; prog[tid >> 6] = 0; }
    }
#endif
    __syncthreads();
    TR_STAMP(1);
    int partner = -1;                                        // the other wave on this wave's SIMD
#if AZ_TOWER_ADAPT
    if constexpr (F == 256) {
        const int me = __builtin_amdgcn_readfirstlane(tid >> 6);
        int nsame = 0;
        for (int i = 0; i < NT / 64; i++)
            if (i != me && prog[8 + i] == prog[8 + me]) { partner = i; nsame++; }
        if (nsame != 1) partner = -1;                        // not exactly two waves on the SIMD
        partner = __builtin_amdgcn_readfirstlane(partner);
    }
#endif
    {
        uint4 wr0[RingPF<1>::PF][NCO];
        ring_fill<1, F, NCO>(wr0, ta.w[0], cw, lane);
        conv_lds<32, RSI, F, RSF, BPW, NCO, false>(ldsb, X, XSZ * 16, zero_off, ta.w[0], nullptr, ta.b[0], wr0, cw,
                                                   bw, lane, wpar, ta.wbytes[0], 0u);
    }
    TR_STAMP(2);
    uint4 wr[RingPF<F / 32>::PF][NCO];
    if (ta.blocks > 0) ring_fill<F / 32, F, NCO>(wr, ta.w[1], cw, lane);
    for (int b = 0; b < ta.blocks; b++) {
        const uint4* after = b + 1 < ta.blocks ? ta.w[3 + 2 * b] : nullptr;
        const unsigned after_bytes = b + 1 < ta.blocks ? ta.wbytes[3 + 2 * b] : 0u;
#ifdef AZ_TOWER_TRACE
        unsigned long long* trw = b == (ta.blocks > 10 ? 10 : ta.blocks - 1) ? ta.trace + (size_t)blockIdx.x * TR_SLOTS + 48 + w * 8 : nullptr;
#else
        unsigned long long* trw = nullptr;
#endif
        conv_lds<F, RSF, F, RSF, BPW, NCO, false, NSP>(ldsb, H, 0, zero_off, ta.w[1 + 2 * b], ta.w[2 + 2 * b],
                                                       ta.b[1 + 2 * b], wr, cw, bw, lane, wpar, ta.wbytes[1 + 2 * b],
                                                       ta.wbytes[2 + 2 * b], trw, done, 1 + 2 * b,
                                                       prog, w, partner);
        conv_lds<F, RSF, F, RSF, BPW, NCO, true, NSP>(ldsb, X, XSZ * 16, zero_off, ta.w[2 + 2 * b], after,
                                                      ta.b[2 + 2 * b], wr, cw, bw, lane, wpar, ta.wbytes[2 + 2 * b],
                                                      after_bytes, trw ? trw + 4 : nullptr, done, 2 + 2 * b, prog, w,
                                                      partner);
        TR_STAMP(3 + b);
    }
    if constexpr (NSP > 1) __syncthreads();           // the heads read every channel
    // heads: NB boards at a time, scratch in H
    {
        constexpr int NB = HeadsCfg<F>::NB;
        static_assert(HeadsScratch<NB, NT>::FLOATS * 4 <= HSZ * 16, "heads scratch must fit in h");
        static_assert((16 * NB) % (NT / 64) == 0, "policy tiles must divide over the waves");
        for (int b0 = 0; b0 < BPB && b0 < nb; b0 += NB)
            heads_group<F, RSF, NB, NT, SEARCH>(ldsb, reinterpret_cast<float*>(H), b0, nb, row0, tid, ta.head_frag,
                                                ta.head, pol_out, val_out, so,
#ifdef AZ_TOWER_TRACE
                                                b0 == 0 ? ta.trace + (size_t)blockIdx.x * TR_SLOTS + 122 : nullptr
#else
                                                nullptr
#endif
            );
    }
    TR_STAMP(45);
#ifdef AZ_TOWER_TRACE
    if (tid == 0) ta.trace[(size_t)blockIdx.x * TR_SLOTS + 113] = __builtin_amdgcn_s_memtime();
#endif
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
#ifndef AZ_T32_NCO256
#define AZ_T32_NCO256 2    // F = 256: 16-channel output fragments per wave (2 = 8 waves, 2 per SIMD; 4 = 4 waves)
#endif
template <int F> struct Tower32Cfg;
template <> struct Tower32Cfg<256> { static constexpr int BPB = 1, WB = 1, NCO = AZ_T32_NCO256; };
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
                                                   ta.head_frag32, ta.head, pol_out, val_out, so, nullptr);
}


// ====================================================================== f32 Winograd tower
// tower32w_kernel: the same f32 tower with every residual 3x3 conv as Winograd F(2x2, 3x3)
// (Lavin & Gray): the 8x8 board is 16 output tiles of 2x2 whose 4x4 input patches are
// transformed V = B^T d B (16 points xi), the weights were transformed on the host
// U = G g G^T (f64, rounded once to f32), M[xi] = U[xi] V[xi] summed over the input channels is
// 16 GEMMs of 256 x 16 tiles x 256 on v_mfma_f32_16x16x4_f32 (exact f32 products), and
// Y = A^T M A.  2.25x fewer MFMAs than the direct conv (16 tiles x 16 points vs 64 squares x 9
// taps).  Numerics: f32 throughout; the transforms' rounding adds ~1.3x the direct f32 error
// (numpy check), checked against the oracle within the f32 tolerance.
// Layout (one board per workgroup, 8 waves of 32 output channels = all 16 points):
//   ACT [64 squares][66 slots] f32 in LDS -- the layer input, overwritten in place by the output
//       (the block input x stays in the registers of the wave that owns it, as the residual);
//   V   2 x [16 xi][8 channel quads][16 tiles][4] f32 = 2 x 32 KB, double-buffered by 32-channel
//       chunks: chunk c+1 is transformed (one (channel, tile) per thread) while the MFMAs of
//       chunk c run; one barrier per chunk;
//   weights [16 ci/16][16 xi][16 co/16][64 lanes][4] f32 per conv, streamed from L2 with a
//       register ring of WINO_PF (xi, 16-channel) steps.
#ifndef AZ_WINO_PF
#define AZ_WINO_PF 2
#endif
#ifndef AZ_WINO_LA
#define AZ_WINO_LA 4
#endif
#ifndef AZ_WINO_TLOAD
#define AZ_WINO_TLOAD 0    // step of a chunk at which the next chunk's patch reads issue
#endif
#ifndef AZ_WINO_TSPLIT
#define AZ_WINO_TSPLIT 2   // steps between the patch reads and their transform + V writes (8 -> 2: C3 tower -1.8 to -2.6 %, profiles/r02_ab_wino_s9_knobs_c3.log)
#endif
#ifndef AZ_WINO_TSTAG
#define AZ_WINO_TSTAG 16   // steps by which the second wave of each SIMD pair (w >= NWV / 2) delays its transform
#endif
#ifndef AZ_WINO_TADDR
#define AZ_WINO_TADDR 1    // 1: patch addresses as per-column bases + immediate row offsets (no per-element multiply)
#endif
constexpr int WINO_TLOAD = AZ_WINO_TLOAD, WINO_TSPLIT = AZ_WINO_TSPLIT, WINO_TSTAG = AZ_WINO_TSTAG;
constexpr int WINO_PF = AZ_WINO_PF;
constexpr int WINO_LA = AZ_WINO_LA;
#ifndef AZ_WINO_NWV
#define AZ_WINO_NWV 8
#endif
#ifndef AZ_WINO_D2
#define AZ_WINO_D2 1       // 1: the patch's row-2 offset as an opaque scalar (no ds_read2st64 pairing, see tload)
#endif
#ifndef AZ_WINO_SWZ
#define AZ_WINO_SWZ 2      // V tile-slot swizzle: slot = tile ^ (SWZ * (quad & 3)); 4 = the round-2 layout (2-way B reads)
#endif
#ifndef AZ_WINO_SYNC
#define AZ_WINO_SYNC 0     // experiment: a workgroup barrier every N steps of a chunk (0: only the per-chunk barrier)
#endif
#ifndef AZ_WINO_PRIO2
#define AZ_WINO_PRIO2 0    // experiment: progress-based issue priority between the two waves of a SIMD
#endif


// Per filter count: NWV waves per workgroup, NN 16-channel output fragments per wave, XH waves per
// output fragment (each on 16 / XH of the Winograd points), XS points per ring step, CH input
// channels per transform chunk (V buffer = CH KB), PF ring steps of weight prefetch.
//   F = 256: 8 waves (two per SIMD) x 32 output channels x all 16 points, one point per step (two
//            independent accumulator chains per step);
//   F = 128: 8 waves x 16 channels x 16 points, two points per step (still two chains: the f32
//            MFMA's dependent latency exceeds its issue interval);
//   F = 64:  8 waves = 4 output fragments x 2 point halves (xi < 8, xi >= 8): two waves per SIMD to
//            share the matrix pipe; A^T M A is linear in M, so each wave transforms its half and the
//            two halves' partial outputs are summed through LDS (2 KB per wave).
template <int F> struct WinoCfg;
#ifndef AZ_WINO64_PF
#define AZ_WINO64_PF 2
#endif
#ifndef AZ_WINO64_CH
#define AZ_WINO64_CH 64    // input channels per transform chunk at F = 64 (64: the whole input in one chunk, C2 A/B -8 %)
#endif
#ifndef AZ_WINO64_XH
#define AZ_WINO64_XH 1     // 1: 4 waves of one point set (with the single 64-channel chunk: C2 tower 102 -> 98.7 us); 2: 8 waves in point halves
#endif
template <> struct WinoCfg<256> {
    static constexpr int NWV = AZ_WINO_NWV, NN = 16 / NWV, XH = 1, XS = 1, CH = 32, PF = WINO_PF;
};
template <> struct WinoCfg<128> { static constexpr int NWV = 8, NN = 1, XH = 1, XS = 2, CH = 32, PF = WINO_PF; };
#ifndef AZ_WINO64_PQ
#define AZ_WINO64_PQ 0     // 1: point quarters (conv_wino_pq: 4 waves x 4 points x all 64 channels, wave-private transforms)
#endif
#ifndef AZ_WINO_PQ_SGB
#define AZ_WINO_PQ_SGB 1   // 1: the point-quarter transform interleaved into the MFMAs by sched_group_barrier
#endif
#if AZ_WINO64_PQ
template <> struct WinoCfg<64> { static constexpr int XH = 4, NWV = 4, NN = 4, XS = 1, CH = 64, PF = 4; };
#else
template <> struct WinoCfg<64> {
    static constexpr int XH = AZ_WINO64_XH, NWV = 4 * XH, NN = 1, XS = 2, CH = AZ_WINO64_CH, PF = AZ_WINO64_PF;
};
#endif
// Winograd weight fragment offsets: wave w's lane base (output fragments NN cw.., its point half) and
// the byte offset of ring step t (16-channel group kl = t / NXI, point t % NXI of the half) of chunk cg
template <int F> __device__ __forceinline__ int wino_voff(int w, int lane) {
    constexpr int NCW = WinoCfg<F>::NWV / WinoCfg<F>::XH, NXI = 16 / WinoCfg<F>::XH, CF = F / 16;
    return (WinoCfg<F>::NN * (w % NCW) * 64 + lane) * 16 + (w / NCW) * NXI * CF * 1024;
}
template <int F> __device__ __forceinline__ int wino_toff(int cg, int t) {
    constexpr int NXI = 16 / WinoCfg<F>::XH, KPC = WinoCfg<F>::CH / 16, CF = F / 16;
    return ((cg * KPC + t / NXI) * 16 + t % NXI) * CF * 1024;
}

// wr: the weight ring; holds this conv's first WINO_PF steps on entry and the next conv's (rN)
// on exit, so no layer starts on a cold weight fetch
template <int F, bool RESID>
__device__ __forceinline__ void conv_wino(char* __restrict__ ldsb, int vbase, int zero_off,
                                          const __amdgpu_buffer_rsrc_t rW, const __amdgpu_buffer_rsrc_t rN,
                                          const float* __restrict__ bias,
                                          f32x4 (&wr)[WinoCfg<F>::PF][WinoCfg<F>::XS][WinoCfg<F>::NN],
                                          f32x4 (&xres)[WinoCfg<F>::NN][4], int w, int lane,
                                          unsigned long long* trw = nullptr) {
    // trw (experiment, -DAZ_WINO_TRACE): s_memtime stamps of this wave: [0] entry, [1] after the
    // prologue barrier, [2 + 2c] chunk c's MFMAs issued, [3 + 2c] after its barrier, [18] epilogue done, [19] exit
#define WT_STAMP(k) do { if (trw && lane == 0) trw[k] = __builtin_amdgcn_s_memtime(); } while (0)
    constexpr int CF = F / 16, RS = F / 4 + 2;
    constexpr int NWV = WinoCfg<F>::NWV, NN = WinoCfg<F>::NN, XS = WinoCfg<F>::XS, XH = WinoCfg<F>::XH;
    constexpr int CH = WinoCfg<F>::CH, VBYTES = CH * 1024, XST = CH * 64;   // V buffer, xi stride
    constexpr int IT = CH * 16 / (NWV * 64);                       // transform items per thread per chunk
    constexpr int NXI = 16 / XH, NCW = NWV / XH;                    // points per wave, output-fragment waves
    // t = (16-channel group kl, point xi0 + t % NXI) pairs of this wave per chunk; a ring step covers XS
    constexpr int NCHUNK = F / CH, KPC = CH / 16, SPC = KPC * NXI, SPX = SPC / XS;
    constexpr int PF = WinoCfg<F>::PF, LA = WINO_LA * XS;
    static_assert(NN * 16 * NCW == F && IT * NWV * 64 == CH * 16 && NWV % 4 == 0 && IT >= 1, "Winograd config");
    static_assert(SPX % PF == 0 && SPC % LA == 0 && NXI % XS == 0, "ring slots must be compile-time");
    const int cw = w % NCW, xp = w / NCW, xi0 = xp * NXI;        // output fragments NN cw.., point half xp
    const int l16 = lane & 15, h = lane >> 4;
    const int ty = l16 >> 2, tx = l16 & 3;
    // V[xi][quad cq][tile slot][4]: tile slot = tile ^ 2 (cq & 3).  gfx950 services a ds_read_b128
    // in the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): each group holds quads h and
    // h + 1 of a fragment at complementary tile sets, and the XOR by 2h keeps their 16 slots distinct
    // (64 banks); a ds_write_b32 of the transform (32-lane groups, 32 banks) then covers 8 distinct
    // slot values mod 8, so both are conflict-free (the earlier XOR by 4h, laid out for groups of 16
    // consecutive lanes, made every B-fragment read 2-way: PMC 48 % of LDS cycles were conflicts)
    const int vrd = h * 256 + ((l16 ^ (AZ_WINO_SWZ * h)) * 16);    // + xi * XST + k * 1024 (cq = 4k + h, cq & 3 = h)
    // transform items: wave w covers tile row ty = w & 3 and 16 channels per item: channel
    // 16 (w >> 2 + it NWV / 4) + (lane & 15) of the chunk, tile (w & 3, lane >> 4) -- a patch read
    // then touches 4 tiles of one row x 16 consecutive channels: conflict-free with the ACT row
    // stride of 8 banks mod 64
    const int tty = w & 3, ttx = lane >> 4;
    auto tchan = [&](int it) { return 16 * ((w >> 2) + it * (NWV / 4)) + (lane & 15); };
    auto vwr = [&](int tch) {   // + xi * XST
        return (tch >> 2) * 256 + (((4 * tty + ttx) ^ (AZ_WINO_SWZ * ((tch >> 2) & 3))) * 16) + (tch & 3) * 4;
    };
    // V[buf] <- B^T d B of chunk c for this thread's item, in two halves: tload issues the patch
    // reads, tstore (WINO_TSPLIT steps later, their latency hidden behind MFMAs) transforms and writes
    auto tload = [&](int c, float (&d)[IT][4][4]) {
        // patch addresses recomputed per chunk from a laundered index: hoisted out of the chunk
        // loop they were 16 loop-invariant registers, and spilled
        const int tl = vgpr_index(ttx);
#if AZ_WINO_TADDR
        // element (i, j) of the patch is square (2 tty - 1 + i, 2 tl - 1 + j): the row part is
        // wave-uniform (tty = w & 3), so every address is a per-column lane base + a row offset
        // that is an instruction immediate (rows 1, 2) or one scalar add (rows 0, 3, clamped onto
        // the board when they fall off it); off-board elements are read at an on-board square and
        // zeroed afterwards (row: wave-uniform select, column: lane select)
        constexpr int R16 = RS * 16;
        const int rowb1 = (2 * tty) * 8 * R16;                              // row i = 1
        const int d0 = tty > 0 ? -8 * R16 : 0, d3 = tty < 3 ? 16 * R16 : 8 * R16;
        // row 2's offset as an opaque scalar: as an immediate the compiler pairs rows 1 and 2 into
        // ds_read2st64_b32 and then moves the pairs apart, waiting for the reads on the spot
        // (s_waitcnt in the step that issues them) instead of steps later in tstore
#if AZ_WINO_D2
        const int d2 = __builtin_amdgcn_readfirstlane(vgpr_index(8 * R16));
#else
        constexpr int d2 = 8 * R16;
#endif
        const bool c0ok = tl > 0, c3ok = tl < 3;
        // the clamped columns (3, 4) keep the 32-lane groups of each ds_read_b32 on distinct banks
        const int cs0 = c0ok ? 2 * tl - 1 : 3, cs3 = c3ok ? 2 * tl + 2 : 4;
#pragma unroll
        for (int it = 0; it < IT; it++) {
            const int chan = (c * CH + tchan(it)) * 4 + rowb1;
            const int cb[4] = {cs0 * R16 + chan, 2 * tl * R16 + chan, (2 * tl + 1) * R16 + chan, cs3 * R16 + chan};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                d[it][0][j] = *reinterpret_cast<const float*>(ldsb + cb[j] + d0);
                d[it][1][j] = *reinterpret_cast<const float*>(ldsb + cb[j]);
                d[it][2][j] = *reinterpret_cast<const float*>(ldsb + cb[j] + d2);
                d[it][3][j] = *reinterpret_cast<const float*>(ldsb + cb[j] + d3);
            }
        }
#else
        const int pty = 2 * tty - 1, ptx = 2 * tl - 1;
#pragma unroll
        for (int it = 0; it < IT; it++) {
            const int chan = (c * CH + tchan(it)) * 4;
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int py = pty + i, px = ptx + j;
                    const bool ok = (unsigned)py < 8u && (unsigned)px < 8u;
                    d[it][i][j] = *reinterpret_cast<const float*>(ldsb + (ok ? (py * 8 + px) * RS * 16 : zero_off) + chan);
                }
        }
#endif
    };
    auto tstore = [&](int buf, const float (&d)[IT][4][4]) {
#if AZ_WINO_TADDR
        const int tl = vgpr_index(ttx);
#endif
#pragma unroll
        for (int it = 0; it < IT; it++) {
            float e[4][4];
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    e[i][j] = d[it][i][j];
#if AZ_WINO_TADDR   // zero the off-board elements tload read at clamped squares
                    if ((i == 0 && tty == 0) || (i == 3 && tty == 3)) e[i][j] = 0.f;
                    if (j == 0) e[i][j] = tl > 0 ? e[i][j] : 0.f;
                    if (j == 3) e[i][j] = tl < 3 ? e[i][j] : 0.f;
#endif
                }
            float t[4][4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                t[0][j] = e[0][j] - e[2][j];
                t[1][j] = e[1][j] + e[2][j];
                t[2][j] = e[2][j] - e[1][j];
                t[3][j] = e[1][j] - e[3][j];
            }
            char* vb = ldsb + vbase + buf * VBYTES + vwr(tchan(it));
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float v0 = t[r][0] - t[r][2], v1 = t[r][1] + t[r][2], v2 = t[r][2] - t[r][1], v3 = t[r][1] - t[r][3];
                *reinterpret_cast<float*>(vb + (r * 4 + 0) * XST) = v0;
                *reinterpret_cast<float*>(vb + (r * 4 + 1) * XST) = v1;
                *reinterpret_cast<float*>(vb + (r * 4 + 2) * XST) = v2;
                *reinterpret_cast<float*>(vb + (r * 4 + 3) * XST) = v3;
            }
        }
    };
    // the residual: this wave's outputs of the block input, read before it is overwritten
    const int co0 = cw * 16 * NN + h * 4;
    auto out_addr = [&](int n, int a, int b) { return ((2 * ty + a) * 8 + 2 * tx + b) * RS * 16 + (co0 + n * 16) * 4; };
    if constexpr (!RESID) {
#pragma unroll
        for (int n = 0; n < NN; n++)
#pragma unroll
            for (int q = 0; q < 4; q++) xres[n][q] = *reinterpret_cast<const f32x4*>(ldsb + out_addr(n, q >> 1, q & 1));
    }
    WT_STAMP(0);
    f32x4 acc[NXI][NN];
#pragma unroll
    for (int x = 0; x < NXI; x++)
#pragma unroll
        for (int n = 0; n < NN; n++) acc[x][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // weight ring: fragment (16-channel group kc, point xi, co/16 = NN cw + n) at ((kc 16 + xi) CF + co/16) KB
    const int voff = wino_voff<F>(w, lane);
    {
        float d0[IT][4][4];
        tload(0, d0);
        tstore(0, d0);
    }
    __syncthreads();
    WT_STAMP(1);
#if AZ_WINO_PRIO2
    __shared__ int prog[NWV];
    int prog_other = 0;
#endif
#pragma unroll 1
    for (int c = 0; c < NCHUNK; c++) {
        float dn[IT][4][4];
        const int vb = vbase + (c & 1) * VBYTES + vrd + xi0 * XST;   // this wave's points
        // B fragment of this wave's step t: 16-channel group t / NXI of the chunk, point xi0 + t % NXI
        auto boff = [](int t) { return (t / NXI) * 1024 + (t % NXI) * XST; };
        const bool more = c + 1 < NCHUNK;
        f32x4 bq[LA];
#pragma unroll
        for (int i = 0; i < LA; i++) bq[i] = *reinterpret_cast<const f32x4*>(ldsb + vb + boff(i));
#pragma unroll
        for (int st = 0; st < SPX; st++) {
            f32x4 B[XS];
#pragma unroll
            for (int xs = 0; xs < XS; xs++) {
                const int t = st * XS + xs;
                B[xs] = bq[t % LA];
                if (t + LA < SPC) {
                    const int s2 = t + LA;
                    bq[t % LA] = *reinterpret_cast<const f32x4*>(ldsb + vb + boff(s2));
                }
            }
            f32x4 a[XS][NN];
#pragma unroll
            for (int xs = 0; xs < XS; xs++)
#pragma unroll
                for (int n = 0; n < NN; n++) a[xs][n] = wr[st % PF][xs][n];
            {
                // ring step st + PF: chunk c (+1 past this chunk's end); past this conv's last
                // step the refills read the next conv's first steps
                const int cadd = (st + PF) / SPX, sl = (st + PF) % SPX;
                const bool nxt = cadd > 0 && !more;
                if constexpr (XH == 1) {
                    // one point set: the steps of a conv are linear in the weights
                    const int tn = c * SPX + st + PF;
                    const int to = (nxt ? tn - NCHUNK * SPX : tn) * XS;
#pragma unroll
                    for (int xs = 0; xs < XS; xs++)
#pragma unroll
                        for (int n = 0; n < NN; n++)
                            wr[st % PF][xs][n] = __builtin_bit_cast(
                                f32x4, __builtin_amdgcn_raw_buffer_load_b128(nxt ? rN : rW,
                                                                             voff + n * 1024 + (to + xs) * CF * 1024, 0, 0));
                } else {
                    const int cg = nxt ? 0 : c + cadd;
#pragma unroll
                    for (int xs = 0; xs < XS; xs++)
#pragma unroll
                        for (int n = 0; n < NN; n++)
                            wr[st % PF][xs][n] = __builtin_bit_cast(
                                f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           nxt ? rN : rW, voff + n * 1024 + wino_toff<F>(cg, sl * XS + xs), 0, 0));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int xs = 0; xs < XS; xs++)
#pragma unroll
                    for (int n = 0; n < NN; n++) {
                        const int x = (st * XS + xs) % NXI;
                        acc[x][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[xs][n][s4], B[xs][s4], acc[x][n], 0, 0, 0);
                    }
            __builtin_amdgcn_sched_barrier(0);
#ifdef AZ_WINO_TRACE
            if (c == 3 && (st & 7) == 7) WT_STAMP(20 + (st >> 3));   // chunk 3, after steps 7, 15, 23, 31
#endif
#if AZ_WINO_SYNC > 0   // experiment: extra workgroup barriers inside a chunk (bounds the skew of a SIMD's two waves)
            if ((st + 1) % AZ_WINO_SYNC == 0 && st + 1 < SPX) __syncthreads();
#endif
#if AZ_WINO_PRIO2   // experiment: every 4 steps the wave behind its SIMD partner (w ^ NWV/2) takes issue priority
            if ((st & 3) == 3) {
                // the partner's progress was read at the previous check (its latency is long past)
                const int mine = c * SPX + st, other = __builtin_amdgcn_readfirstlane(prog_other);
                if (other < mine) __builtin_amdgcn_s_setprio(0);
                else __builtin_amdgcn_s_setprio(1);
                prog[w] = mine;
                prog_other = prog[w ^ (NWV / 2)];
            }
#endif
#ifndef AZ_WINO_NOTRANSFORM   // experiment only: no input transforms inside the chunk loop (wrong results)
            // (a stagger that would not fit in this F's chunk is dropped)
            constexpr int TSG = (WINO_TLOAD + WINO_TSTAG + WINO_TSPLIT) / XS < SPX ? WINO_TSTAG : 0;
            if constexpr (TSG == 0) {
                if (st == WINO_TLOAD / XS && more) tload(c + 1, dn);
                if (st == (WINO_TLOAD + WINO_TSPLIT) / XS && more) tstore((c + 1) & 1, dn);
            } else {
                // the two waves of a SIMD pair run their transform VALU blocks at different steps,
                // so that one of them keeps the matrix pipe busy
                const bool late = w >= NWV / 2;
                if (st == WINO_TLOAD / XS && more && !late) tload(c + 1, dn);
                if (st == (WINO_TLOAD + TSG) / XS && more && late) tload(c + 1, dn);
                if (st == (WINO_TLOAD + WINO_TSPLIT) / XS && more && !late) tstore((c + 1) & 1, dn);
                if (st == (WINO_TLOAD + TSG + WINO_TSPLIT) / XS && more && late) tstore((c + 1) & 1, dn);
            }
#endif
        }
        WT_STAMP(2 + 2 * c);
        __syncthreads();
        WT_STAMP(3 + 2 * c);
    }
    // output transform Y = A^T M A per (output fragment n, channel r), + bias (+ residual), ReLU
    if constexpr (XH == 1) {
#pragma unroll
        for (int n = 0; n < NN; n++) {
            const float4 bb = *reinterpret_cast<const float4*>(bias + co0 + n * 16);
            f32x4 y[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float m[4][4];
#pragma unroll
                for (int x = 0; x < 16; x++) m[x >> 2][x & 3] = acc[x][n][r];
                float s0[4], s1[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    s0[j] = m[0][j] + m[1][j] + m[2][j];
                    s1[j] = m[1][j] - m[2][j] - m[3][j];
                }
                const float br = r == 0 ? bb.x : r == 1 ? bb.y : r == 2 ? bb.z : bb.w;
                y[0][r] = (s0[0] + s0[1] + s0[2]) + br;
                y[1][r] = (s0[1] - s0[2] - s0[3]) + br;
                y[2][r] = (s1[0] + s1[1] + s1[2]) + br;
                y[3][r] = (s1[1] - s1[2] - s1[3]) + br;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                f32x4 v = y[q];
                if constexpr (RESID) v += xres[n][q];
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = fmaxf(v[r], 0.0f);
                *reinterpret_cast<f32x4*>(ldsb + out_addr(n, q >> 1, q & 1)) = v;
            }
        }
    } else {
        // two point halves: this wave holds rows a = 2 xp, 2 xp + 1 of M (xi = 4 a + b); its partial
        // A^T M A, then the half-output of the partner's two channels goes through V (free after the
        // last chunk's barrier) and this wave finishes channels 2 xp, 2 xp + 1 of its fragment
        static_assert(XH == 2 && NN == 1, "point halves: one output fragment per wave");
        f32x4 y[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float s0[4], s1[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float m0 = acc[j][0][r], m1 = acc[4 + j][0][r];
                s0[j] = xp ? m0 : m0 + m1;                    // A^T row 0 = [1 1 1 0]
                s1[j] = xp ? -(m0 + m1) : m1;                 // A^T row 1 = [0 1 -1 -1]
            }
            y[0][r] = s0[0] + s0[1] + s0[2];
            y[1][r] = s0[1] - s0[2] - s0[3];
            y[2][r] = s1[0] + s1[1] + s1[2];
            y[3][r] = s1[1] - s1[2] - s1[3];
        }
        // send channels 2 (1 - xp) + {0, 1}: [q][2] as two 16-byte writes
        const int ro = xp ? 0 : 2;
        char* xb = ldsb + vbase + ((cw * 2 + (1 - xp)) * 64 + lane) * 32;
        *reinterpret_cast<f32x4*>(xb) = f32x4{y[0][ro], y[0][ro + 1], y[1][ro], y[1][ro + 1]};
        *reinterpret_cast<f32x4*>(xb + 16) = f32x4{y[2][ro], y[2][ro + 1], y[3][ro], y[3][ro + 1]};
        __syncthreads();
        const char* rb = ldsb + vbase + ((cw * 2 + xp) * 64 + lane) * 32;
        const f32x4 g0 = *reinterpret_cast<const f32x4*>(rb), g1 = *reinterpret_cast<const f32x4*>(rb + 16);
        const float recv[4][2] = {{g0[0], g0[1]}, {g0[2], g0[3]}, {g1[0], g1[1]}, {g1[2], g1[3]}};
        const int rk = xp ? 2 : 0;
        const float2 bb = *reinterpret_cast<const float2*>(bias + co0 + rk);
        typedef __attribute__((ext_vector_type(2))) float f32x2;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            f32x2 v;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const float own = xp ? y[q][2 + i] : y[q][i];
                v[i] = (own + recv[q][i]) + (i ? bb.y : bb.x);
                if constexpr (RESID) v[i] += xp ? xres[0][q][2 + i] : xres[0][q][i];
                v[i] = fmaxf(v[i], 0.0f);
            }
            *reinterpret_cast<f32x2*>(ldsb + out_addr(0, q >> 1, q & 1) + rk * 4) = v;
        }
    }
    WT_STAMP(18);
    __syncthreads();
    WT_STAMP(19);
#undef WT_STAMP
}

// Point quarters (F = 64, one board, 4 waves = one per SIMD): wave w owns the Winograd points
// xi = 4w..4w+3 (row w of the 4x4 point grid) for all F output channels.  Row w of B^T d B needs
// two patch rows, so each wave transforms only its own points into a wave-private V region: its
// transform and its MFMAs need no workgroup barrier, and the transform of 16-channel group kc+1
// runs under the MFMAs of group kc.  A^T M A needs all 16 points of a (channel, tile): every wave
// passes its M rows through its V region (one barrier) and wave n finishes output fragment n with
// the one-point-set kernel's arithmetic in the same order, so M and the outputs are bit-identical
// to WinoCfg<64>{XH = 1} (the transforms compute the same rows, the MFMAs accumulate each point
// over kc and s4 in the same order).  LDS: V region w = [kc 4][point 4][quad 4][tile slot 16][4]
// f32 = 16 KB, reused for the M exchange ([fragment 4][point 4][64 lanes][4]).
// wr: the weight ring, [PF steps][1][4 fragments]; step s = (kc = s / 4, point 4w + s % 4).
template <int F, bool RESID>
__device__ __forceinline__ void conv_wino_pq(char* __restrict__ ldsb, int vbase, const __amdgpu_buffer_rsrc_t rW,
                                             const __amdgpu_buffer_rsrc_t rN, const float* __restrict__ bias,
                                             f32x4 (&wr)[WinoCfg<F>::PF][1][WinoCfg<F>::NN],
                                             f32x4 (&xres)[WinoCfg<F>::NN][4], int w, int lane) {
    constexpr int CF = F / 16, RS = F / 4 + 2, R16 = RS * 16;
    constexpr int NN = WinoCfg<F>::NN, PF = WinoCfg<F>::PF, NKC = F / 16, NST = NKC * 4;
    static_assert(NN == CF && WinoCfg<F>::NWV == 4 && WinoCfg<F>::XS == 1 && NST % PF == 0, "point quarters");
    const int l16 = lane & 15, h = lane >> 4;
    const int ty = l16 >> 2, tx = l16 & 3;
    const int vw = vbase + w * (NKC * 4096);                   // this wave's V region
    // transform items: channel lane & 15 of the group, tile (it, lane >> 4), it = 0..3
    const int tch = lane & 15, ttx = vgpr_index(lane >> 4);
    // this wave's row of B^T: t = d[ra] + d[rb] (w = 1) or d[ra] - d[rb]
    const int ra = w == 0 ? 0 : w == 2 ? 2 : 1, rb = w == 0 ? 2 : w == 1 ? 2 : w == 2 ? 1 : 3;
    const bool tadd = w == 1;
    // columns of the patch; off-board ones read the clamped columns 3 / 4 (distinct banks within
    // each 32-lane group, as in conv_wino) and are zeroed
    const int cs0 = ttx > 0 ? 2 * ttx - 1 : 3, cs3 = ttx < 3 ? 2 * ttx + 2 : 4;
    const int ccol[4] = {cs0 * R16, 2 * ttx * R16, (2 * ttx + 1) * R16, cs3 * R16};
    auto tload = [&](int kc, float (&d)[4][2][4]) {
        const int chan = (kc * 16 + tch) * 4;
#pragma unroll
        for (int it = 0; it < 4; it++) {
            // patch rows 2 it - 1 + ra / rb, clamped onto the board (zeroed in tstore)
            const int pa = min(max(2 * it - 1 + ra, 0), 7), pb = min(max(2 * it - 1 + rb, 0), 7);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                d[it][0][j] = *reinterpret_cast<const float*>(ldsb + pa * 8 * R16 + ccol[j] + chan);
                d[it][1][j] = *reinterpret_cast<const float*>(ldsb + pb * 8 * R16 + ccol[j] + chan);
            }
        }
    };
    auto tstore = [&](int kc, const float (&d)[4][2][4]) {
        const int quad = tch >> 2;
        char* vb = ldsb + vw + kc * 4096 + quad * 256 + (tch & 3) * 4;
#pragma unroll
        for (int it = 0; it < 4; it++) {
            const bool oka = (unsigned)(2 * it - 1 + ra) < 8u, okb = (unsigned)(2 * it - 1 + rb) < 8u;
            float t[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool okc = j == 0 ? ttx > 0 : j == 3 ? ttx < 3 : true;
                const float ea = oka && okc ? d[it][0][j] : 0.f, eb = okb && okc ? d[it][1][j] : 0.f;
                t[j] = tadd ? ea + eb : ea - eb;
            }
            const float v[4] = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
            const int slot = ((4 * it + ttx) ^ (AZ_WINO_SWZ * (quad & 3))) * 16;
#pragma unroll
            for (int c = 0; c < 4; c++) *reinterpret_cast<float*>(vb + c * 1024 + slot) = v[c];
        }
    };
    // B fragment of step s: group s / 4, point 4w + s % 4 (the conv_wino V layout, one point set)
    const int vrd = vw + h * 256 + ((l16 ^ (AZ_WINO_SWZ * h)) * 16);
    auto bread = [&](int s) { return *reinterpret_cast<const f32x4*>(ldsb + vrd + (s >> 2) * 4096 + (s & 3) * 1024); };
    const int co0 = w * 16 + h * 4;                              // the fragment this wave finishes
    auto out_addr = [&](int a, int b) { return ((2 * ty + a) * 8 + 2 * tx + b) * R16 + co0 * 4; };
    if constexpr (!RESID) {
#pragma unroll
        for (int q = 0; q < 4; q++) xres[0][q] = *reinterpret_cast<const f32x4*>(ldsb + out_addr(q >> 1, q & 1));
    }
    f32x4 acc[4][NN];
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int n = 0; n < NN; n++) acc[x][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int voff = lane * 16 + 4 * w * CF * 1024;
    float dn[4][2][4];
    tload(0, dn);
    tstore(0, dn);
    // the V region is this wave's own: program order (LDS executes a wave's operations in order)
    // is the only hand-off, the fence keeps the compiler from moving the reads above the writes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    f32x4 Bc = bread(0);
#pragma unroll
    for (int s = 0; s < NST; s++) {
        const int kc = s >> 2, j = s & 3;
        const bool more = kc + 1 < NKC;
        f32x4 Bn = Bc;
        if (s + 1 < NST) Bn = bread(s + 1);
        f32x4 a[NN];
#pragma unroll
        for (int n = 0; n < NN; n++) a[n] = wr[s % PF][0][n];
        {   // refill with step s + PF (past this conv's end: the next conv's first steps)
            const int tn = s + PF;
            const bool nxt = tn >= NST;
            const int t2 = nxt ? tn - NST : tn;
            const int to = ((t2 >> 2) * 16 + (t2 & 3)) * CF * 1024;
#pragma unroll
            for (int n = 0; n < NN; n++)
                wr[s % PF][0][n] = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(nxt ? rN : rW, voff + n * 1024 + to, 0, 0));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
            for (int n = 0; n < NN; n++) acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[n][s4], Bc[s4], acc[j][n], 0, 0, 0);
        // one wave per SIMD: the next group's transform must issue between this step's MFMAs (a
        // VALU or LDS instruction issues in the shadow of a 32-cycle MFMA), not after them
        if (j == 0 && more) tload(kc + 1, dn);
        if (j == 1 && more) tstore(kc + 1, dn);
#if AZ_WINO_PQ_SGB
        if (j == 0 && more) {
#pragma unroll
            for (int i = 0; i < 4 * NN; i++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS read
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);   // VALU
            }
        }
        if (j == 1 && more) {
#pragma unroll
            for (int i = 0; i < 4 * NN; i++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);   // VALU
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // DS write
            }
        }
#endif
        __builtin_amdgcn_sched_barrier(0);
        if (j == 1 && more) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        Bc = Bn;
    }
    // M exchange: [fragment n][point j][lane] in this wave's V region (its own reads are done:
    // in order), then wave n gathers fragment n's 16 points from the 4 regions
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int n = 0; n < NN; n++)
#pragma unroll
        for (int j = 0; j < 4; j++) *reinterpret_cast<f32x4*>(ldsb + vw + (n * 4 + j) * 1024 + lane * 16) = acc[j][n];
    __syncthreads();
    f32x4 m16[16];
#pragma unroll
    for (int x = 0; x < 16; x++)
        m16[x] = *reinterpret_cast<const f32x4*>(ldsb + vbase + (x >> 2) * (NKC * 4096) + (w * 4 + (x & 3)) * 1024 + lane * 16);
    {
        const float4 bb = *reinterpret_cast<const float4*>(bias + co0);
        f32x4 y[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float m[4][4];
#pragma unroll
            for (int x = 0; x < 16; x++) m[x >> 2][x & 3] = m16[x][r];
            float s0[4], s1[4];
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                s0[jj] = m[0][jj] + m[1][jj] + m[2][jj];
                s1[jj] = m[1][jj] - m[2][jj] - m[3][jj];
            }
            const float br = r == 0 ? bb.x : r == 1 ? bb.y : r == 2 ? bb.z : bb.w;
            y[0][r] = (s0[0] + s0[1] + s0[2]) + br;
            y[1][r] = (s0[1] - s0[2] - s0[3]) + br;
            y[2][r] = (s1[0] + s1[1] + s1[2]) + br;
            y[3][r] = (s1[1] - s1[2] - s1[3]) + br;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            f32x4 v = y[q];
            if constexpr (RESID) v += xres[0][q];
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = fmaxf(v[r], 0.0f);
            *reinterpret_cast<f32x4*>(ldsb + out_addr(q >> 1, q & 1)) = v;
        }
    }
    __syncthreads();
}

// ====================================================================== F = 256: per-wave transforms
// conv_wino_dt: the 256-filter Winograd conv with NO shared transform buffer and no barrier inside
// the conv.  Each of the 8 waves (2 per SIMD) owns 32 output channels x all 16 points x all 16
// tiles (128 accumulators) and computes the input transform V = B^T d B it needs ITSELF, in
// registers, straight in the MFMA B layout: lane (h, tile) transforms channel 4t + h of its tile
// for input quarter t (4 channels), from a 4x4 patch read out of the padded activation image.  The
// 8-fold duplicated transform (32 VALU + 16 ds_read_b32 per quarter per wave, against 32 MFMAs)
// runs in the MFMAs' issue shadows, software-pipelined one quarter ahead (two 16-register V slots),
// so a wave's matrix stream never waits on another wave: the round-2 kernel's 8 chunk barriers per
// conv (and the V writes between them) are gone, which is where its 17 % idle matrix pipe went
// (DESIGN.md section 5.4).  Two barriers per conv remain: after the MFMAs (every wave has read the
// layer input) and after the epilogue (the output is the next conv's input).
// LDS (one board): a zero guard, then ACTP -- the layer input f32, rows padded with zero rows
// above and below, 9 squares per row (the 9th is a zero column that is also the left neighbour of
// the next row's first square) and 11 pad words, so every patch element is base + immediate with no
// bounds logic; square stride 257 words and row stride 2324 (= 20 mod 32) make the 32 lanes of each
// ds_read_b32 hit 32 distinct banks (8 ty + 2 tx + h) -- then RES, the block input (the residual of
// conv 2 and, after the tower, the heads' input) in the round-2 layout [64 squares][66 slots].
// Weights [quarter t 64][point quad q 4][co/16 16][lane 64][4 points] f32 (winograd_f32, net.hip):
// one coalesced dwordx4 per lane = 4 points of one (co, ci); an 8-slot register ring (one quarter)
// refilled right after each slot's 4 MFMAs, across conv boundaries.
constexpr int DT_BETA = 257;                     // words per square (256 channels + 1)
constexpr int DT_ALPHA = 2324;                   // words per padded row (9 squares + 11)
constexpr int DT_GUARD = 260;                    // zero words before ACTP (>= DT_BETA: the (-1, -1) neighbour; RES 16-B aligned)
constexpr int DT_ACT_WORDS = 10 * DT_ALPHA;
constexpr int DT_ACT_BYTES = (DT_GUARD + DT_ACT_WORDS) * 4;   // guard + ACTP
constexpr int DT_RES_BYTES = 64 * 66 * 16;                     // RES, the round-2 [64][66 slots] layout
#ifndef AZ_DT_RING
#define AZ_DT_RING 4       // weight-ring slots (f32x4 each) a wave keeps in flight (8 = one input quarter)
#endif
constexpr int DT_RING = AZ_DT_RING;
static_assert(DT_RING == 4 || DT_RING == 8, "ring of half or one quarter");
static_assert(DT_ACT_BYTES % 16 == 0, "RES must start 16-B aligned");

template <bool RESID>
__device__ __forceinline__ void conv_wino_dt(char* __restrict__ ldsb, const __amdgpu_buffer_rsrc_t rW,
                                             const __amdgpu_buffer_rsrc_t rN, const float* __restrict__ bias,
                                             f32x4 (&wr)[DT_RING / 2][2], int w, int lane) {
    constexpr int NQ = 64;                                      // input quarters (4 channels each)
    constexpr int QB = 4 * 16 * 1024;                           // weight bytes per quarter (all co)
    const int l16 = lane & 15, h = lane >> 4;
    const int ty = l16 >> 2, tx = l16 & 3;
    // patch element (r, c) of tile (ty, tx) = square (2ty - 1 + r, 2tx - 1 + c) = padded row 2ty + r,
    // column 2tx - 1 + c (column -1 = the zero column 8 of the row above)
    const int pbase = (DT_GUARD + 2 * ty * DT_ALPHA + (2 * tx - 1) * DT_BETA + h) * 4;
    const int voff = (2 * w * 64 + lane) * 16;
    f32x4 acc[16][2];
#pragma unroll
    for (int x = 0; x < 16; x++)
#pragma unroll
        for (int n = 0; n < 2; n++) acc[x][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float V[2][16];
    // channel 4t + h of the patch: 16 ds_read_b32 at immediate offsets from one lane base
    auto pread = [&](int cbyte, float (&d)[16]) {
        const char* p = ldsb + cbyte;
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++) d[r * 4 + c] = *reinterpret_cast<const float*>(p + (r * DT_ALPHA + c * DT_BETA) * 4);
    };
    // B^T d B in place, the round-2 kernel's operation order (rows first): bit-identical V
    auto transform = [&](float (&d)[16]) {
        float t[4][4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            t[0][j] = d[0 * 4 + j] - d[2 * 4 + j];
            t[1][j] = d[1 * 4 + j] + d[2 * 4 + j];
            t[2][j] = d[2 * 4 + j] - d[1 * 4 + j];
            t[3][j] = d[1 * 4 + j] - d[3 * 4 + j];
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            d[r * 4 + 0] = t[r][0] - t[r][2];
            d[r * 4 + 1] = t[r][1] + t[r][2];
            d[r * 4 + 2] = t[r][2] - t[r][1];
            d[r * 4 + 3] = t[r][1] - t[r][3];
        }
    };
    pread(pbase, V[0]);
    transform(V[0]);
#pragma unroll 1
    for (int g = 0; g < NQ / 4; g++) {
        const int gb = vgpr_index(pbase + g * 64);              // channels 16g + 4j + h
        const bool last = g + 1 == NQ / 4;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int cur = j & 1, nxt = cur ^ 1;
            const bool more = j < 3 || !last;
            // next quarter's patch into the other slot (its V was consumed by the last quarter's MFMAs)
            if (more) pread(j < 3 ? gb + (j + 1) * 16 : gb + 64, V[nxt]);
            // refills: quarter t + 1 of this conv, or quarter 0 of the next one (rN)
            const bool wrap = j == 3 && last;
            const int soff = wrap ? 0 : (j < 3 ? g * 4 + j + 1 : g * 4 + 4) * QB;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int n = 0; n < 2; n++) {
                    // ring slot k = 2q + n holds slot k of this quarter; refilled with slot k + RING of
                    // the sequence (this quarter's later slots, then the next quarter's)
                    const int k = 2 * q + n;
                    const f32x4 a = wr[(k % DT_RING) / 2][(k % DT_RING) % 2];
#pragma unroll
                    for (int p = 0; p < 4; p++)
                        acc[4 * q + p][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[p], V[cur][4 * q + p], acc[4 * q + p][n], 0, 0, 0);
                    const int kn = k + DT_RING;                 // slot of the sequence to fetch
                    const bool nq = kn >= 8;                    // ... in the next quarter
                    const int qs = (kn & 7) / 2, ns = (kn & 7) % 2;
                    const bool use_n = nq && wrap;
                    const int so2 = nq ? soff : (g * 4 + j) * QB;
                    wr[(k % DT_RING) / 2][(k % DT_RING) % 2] = __builtin_bit_cast(
                        f32x4, __builtin_amdgcn_raw_buffer_load_b128(use_n ? rN : rW, voff + (qs * 16 + ns) * 1024, so2, 0));
                }
            if (more) transform(V[nxt]);
            // interleave: per slot (4 MFMAs) one weight refill, the patch reads up front and the next
            // quarter's transform VALU spread over the MFMAs
#ifndef AZ_DT_SGB
#define AZ_DT_SGB 1
#endif
#if AZ_DT_SGB
#pragma unroll
            for (int i = 0; i < 8; i++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);        // 4 MFMAs
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);        // 1 VMEM read (weight refill)
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);        // 4 VALU (transform)
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);        // 2 DS reads (next patch)
            }
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    __syncthreads();                                            // every wave has read the layer input
    // output transform Y = A^T M A, + bias (+ residual from RES), ReLU -> ACTP (and RES after conv 2)
    const int co0 = w * 32 + h * 4;
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const float4 bb = *reinterpret_cast<const float4*>(bias + co0 + n * 16);
        f32x4 y[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float m[4][4];
#pragma unroll
            for (int x = 0; x < 16; x++) m[x >> 2][x & 3] = acc[x][n][r];
            float s0[4], s1[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                s0[j] = m[0][j] + m[1][j] + m[2][j];
                s1[j] = m[1][j] - m[2][j] - m[3][j];
            }
            const float br = r == 0 ? bb.x : r == 1 ? bb.y : r == 2 ? bb.z : bb.w;
            y[0][r] = (s0[0] + s0[1] + s0[2]) + br;
            y[1][r] = (s0[1] - s0[2] - s0[3]) + br;
            y[2][r] = (s1[0] + s1[1] + s1[2]) + br;
            y[3][r] = (s1[1] - s1[2] - s1[3]) + br;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int a = q >> 1, b = q & 1;
            const int co = co0 + n * 16;
            char* rp = ldsb + DT_ACT_BYTES + (((2 * ty + a) * 8 + 2 * tx + b) * 66) * 16 + co * 4;
            f32x4 v = y[q];
            if constexpr (RESID) v += *reinterpret_cast<const f32x4*>(rp);
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = fmaxf(v[r], 0.0f);
            if constexpr (RESID) *reinterpret_cast<f32x4*>(rp) = v;
            float* ap = reinterpret_cast<float*>(ldsb + (DT_GUARD + (2 * ty + a + 1) * DT_ALPHA + (2 * tx + b) * DT_BETA + co) * 4);
#pragma unroll
            for (int r = 0; r < 4; r++) ap[r] = v[r];
        }
    }
    __syncthreads();
}

// one board (batch row row0) through the 256-filter Winograd f32 tower with per-wave transforms
template <bool SEARCH>
__device__ __forceinline__ void tower32w_board_dt(const float* __restrict__ planes, const TowerArgs& ta, int row0,
                                                  float* __restrict__ pol_out, float* __restrict__ val_out,
                                                  const SearchOut& so, int tid) {
    constexpr int F = 256, NT = 512, NN = 2;
    constexpr int RSF = F / 4 + 2, RSI = 32 / 4 + 2;
    constexpr int PLANES_BYTES = 64 * RSI * 16, ZN = 16 + F / 4;
    static_assert(PLANES_BYTES + ZN * 16 <= DT_ACT_BYTES, "input planes + zero row must fit in ACTP");
    static_assert(HeadsScratch<1, NT, heads_npart(NT, true)>::FLOATS * 4 <= DT_ACT_BYTES, "heads scratch must fit in ACTP");
    __shared__ __attribute__((aligned(16))) uint4 lds[(DT_ACT_BYTES + DT_RES_BYTES) / 16];
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    char* ldsb = reinterpret_cast<char*>(lds);
    uint4* RES = lds + DT_ACT_BYTES / 16;
    // input conv 19 (32) -> F, direct f32 (conv32_lds): planes staged at the start of the ACTP
    // region, its zero row behind them, output into RES
    stage_planes_f32<1, RSI, NT>(lds, planes, so, row0, 1, tid);
    for (int c = tid; c < ZN; c += NT) lds[PLANES_BYTES / 16 + c] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    {
        f32x4 wr[T32_PF][NN];
        const __amdgpu_buffer_rsrc_t r0 = t32_rsrc(ta.w[0], ta.wbytes[0]);
        const __amdgpu_buffer_rsrc_t rz = t32_rsrc(ta.w[0] + 18 * (F / 16) * 64, ta.wbytes[0] - 18 * (F / 16) * 1024);
        const int voff = ((w * NN) * 64 + lane) * 16;
#pragma unroll
        for (int i = 0; i < T32_PF; i++)
#pragma unroll
            for (int n = 0; n < NN; n++)
                wr[i][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r0, voff + n * 1024 + i * (F / 16) * 1024, 0, 0));
        conv32_lds<32, RSI, F, RSF, 1, NN, false>(ldsb, reinterpret_cast<char*>(RES), 0, PLANES_BYTES, r0, rz, ta.b[0],
                                                  wr, w, 0, lane);   // ends with a barrier
    }
    // ACTP <- RES: zero the guard, pad rows / column / words, then the 64 squares
    for (int c = tid; c < DT_ACT_BYTES / 16; c += NT) lds[c] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (int c = tid; c < 64 * 64; c += NT) {
        const int sq = c >> 6, q = c & 63;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ldsb + DT_ACT_BYTES + (sq * RSF + q) * 16);
        float* ap = reinterpret_cast<float*>(ldsb + (DT_GUARD + ((sq >> 3) + 1) * DT_ALPHA + (sq & 7) * DT_BETA + 4 * q) * 4);
#pragma unroll
        for (int r = 0; r < 4; r++) ap[r] = v[r];
    }
    __syncthreads();
    f32x4 wring[DT_RING / 2][2];
    if (ta.blocks > 0) {
        const __amdgpu_buffer_rsrc_t r = t32_rsrc(ta.ww[0], ta.wwbytes[0]);
        const int voff = (2 * w * 64 + lane) * 16;
#pragma unroll
        for (int q = 0; q < DT_RING / 2; q++)
#pragma unroll
            for (int n = 0; n < 2; n++)
                wring[q][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + (q * 16 + n) * 1024, 0, 0));
    }
    for (int b = 0; b < ta.blocks; b++) {
        const unsigned wb3 = b + 1 < ta.blocks ? ta.wwbytes[2 * b + 2] : 0u;   // after the last conv: nothing (reads 0)
        const __amdgpu_buffer_rsrc_t r1 = t32_rsrc(ta.ww[2 * b], ta.wwbytes[2 * b]);
        const __amdgpu_buffer_rsrc_t r2 = t32_rsrc(ta.ww[2 * b + 1], ta.wwbytes[2 * b + 1]);
        const __amdgpu_buffer_rsrc_t r3 = t32_rsrc(b + 1 < ta.blocks ? ta.ww[2 * b + 2] : ta.ww[2 * b + 1], wb3);
        conv_wino_dt<false>(ldsb, r1, r2, ta.b[1 + 2 * b], wring, w, lane);
        conv_wino_dt<true>(ldsb, r2, r3, ta.b[2 + 2 * b], wring, w, lane);
    }
    // heads from RES (the last block's output), scratch in the ACTP region
    heads_group<F, RSF, 1, NT, SEARCH, true>(reinterpret_cast<const char*>(RES), reinterpret_cast<float*>(lds), 0, 1,
                                             row0, tid, ta.head_frag32, ta.head, pol_out, val_out, so, nullptr);
}

// one board (batch row row0) through the Winograd f32 tower with transform chunks shared by all NWV
// waves (F = 64, 128; and F = 256 when built with AZ_WINO_DT=0)
template <int F, bool SEARCH>
__device__ __forceinline__ void tower32w_board_shared(const float* __restrict__ planes, const TowerArgs& ta, int row0,
                                                      float* __restrict__ pol_out, float* __restrict__ val_out,
                                                      const SearchOut& so, int tid) {
    constexpr int NWV = WinoCfg<F>::NWV, NT = NWV * 64, NN = WinoCfg<F>::NN, XS = WinoCfg<F>::XS;
    constexpr int XH = WinoCfg<F>::XH, NCW = NWV / XH;    // waves of the direct input conv
    constexpr int RSF = F / 4 + 2, RSI = 32 / 4 + 2;
    constexpr int XSZ = 64 * RSF;                        // ACT, uint4 slots
    // both V buffers (one when a single chunk covers the input), also planes staging / heads scratch
    constexpr int VSZ = (F / WinoCfg<F>::CH > 1 ? 2 : 1) * WinoCfg<F>::CH * 1024 / 16;
    constexpr int PF = WinoCfg<F>::PF;
    constexpr int ZN = 16 + F / 4;
    static_assert(HeadsScratch<1, NT, heads_npart(NT, true)>::FLOATS * 4 <= VSZ * 16, "heads scratch must fit in V");
    static_assert(64 * RSI <= VSZ, "input planes must fit in V");
    __shared__ __attribute__((aligned(16))) uint4 lds[XSZ + VSZ + ZN];
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint4* X = lds;
    uint4* V = lds + XSZ;
    const int vbase = XSZ * 16;
    const int zero_off = (XSZ + VSZ) * 16;
    char* ldsb = reinterpret_cast<char*>(lds);
#ifdef AZ_WINO_TRACE   // coarse per-wave stamps: slots 192 + 16 w + k (k: 0 start, 1 staged, 2 input conv, 3 + b block b, 15 end)
    unsigned long long* trc = w < 4 ? ta.trace + (size_t)blockIdx.x * TR_SLOTS + 192 + 16 * w : nullptr;   // waves 0-3
#define WC_STAMP(k) do { if (trc && lane == 0) trc[k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define WC_STAMP(k) do { } while (0)
#endif
    WC_STAMP(0);
    stage_planes_f32<1, RSI, NT>(V, planes, so, row0, 1, tid);
    for (int c = tid; c < ZN; c += NT) lds[XSZ + VSZ + c] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    WC_STAMP(1);
    {   // input conv 19 (32) -> F: direct (18 k-steps)
        auto input_conv = [&]() {
            f32x4 wr[T32_PF][NN];
            const __amdgpu_buffer_rsrc_t r0 = t32_rsrc(ta.w[0], ta.wbytes[0]);
            const __amdgpu_buffer_rsrc_t rz = t32_rsrc(ta.w[0] + 18 * (F / 16) * 64, ta.wbytes[0] - 18 * (F / 16) * 1024);
            const int voff = ((w * NN) * 64 + lane) * 16;
#pragma unroll
            for (int i = 0; i < T32_PF; i++)
#pragma unroll
                for (int n = 0; n < NN; n++)
                    wr[i][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                             r0, voff + n * 1024 + i * (F / 16) * 1024, 0, 0));
            conv32_lds<32, RSI, F, RSF, 1, NN, false>(ldsb, reinterpret_cast<char*>(X), vbase, zero_off, r0, rz, ta.b[0],
                                                      wr, w, 0, lane);
        };
        if constexpr (XH == 4) {   // point quarters: every wave, one 16-channel fragment each
            f32x4 wr[T32_PF][1];
            const __amdgpu_buffer_rsrc_t r0 = t32_rsrc(ta.w[0], ta.wbytes[0]);
            const __amdgpu_buffer_rsrc_t rz = t32_rsrc(ta.w[0] + 18 * (F / 16) * 64, ta.wbytes[0] - 18 * (F / 16) * 1024);
            const int voff = (w * 64 + lane) * 16;
#pragma unroll
            for (int i = 0; i < T32_PF; i++)
                wr[i][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r0, voff + i * (F / 16) * 1024, 0, 0));
            conv32_lds<32, RSI, F, RSF, 1, 1, false>(ldsb, reinterpret_cast<char*>(X), vbase, zero_off, r0, rz, ta.b[0],
                                                     wr, w, 0, lane);
        } else if constexpr (XH == 1) {
            input_conv();
        } else {   // point halves: only the first NCW waves; the others meet its closing barrier
            if (w < NCW) input_conv();
            else __syncthreads();
        }
    }
#ifdef AZ_WINO_YPRIO   // experiment: the younger wave of each SIMD pair (w >= 4) issues first
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
#endif
    WC_STAMP(2);
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
#ifdef AZ_WINO_TRACE
        unsigned long long* trw = b == (ta.blocks > 10 ? 10 : ta.blocks - 1) ? ta.trace + (size_t)blockIdx.x * TR_SLOTS + w * 24 : nullptr;
#else
        unsigned long long* trw = nullptr;
#endif
#ifdef AZ_WINO_NOWEIGHTS   // experiment only: zero-record descriptors drop every weight load (wrong results)
        const unsigned wb1 = 0, wb2 = 0, wb3 = 0;
#else
        const unsigned wb1 = ta.wwbytes[2 * b], wb2 = ta.wwbytes[2 * b + 1];
        const unsigned wb3 = b + 1 < ta.blocks ? ta.wwbytes[2 * b + 2] : 0u;   // after the last conv: nothing (reads 0)
#endif
        const __amdgpu_buffer_rsrc_t r1 = t32_rsrc(ta.ww[2 * b], wb1), r2 = t32_rsrc(ta.ww[2 * b + 1], wb2);
        const __amdgpu_buffer_rsrc_t r3 = t32_rsrc(b + 1 < ta.blocks ? ta.ww[2 * b + 2] : ta.ww[2 * b + 1], wb3);
        if constexpr (XH == 4) {
            conv_wino_pq<F, false>(ldsb, vbase, r1, r2, ta.b[1 + 2 * b], wring, xres, w, lane);
            conv_wino_pq<F, true>(ldsb, vbase, r2, r3, ta.b[2 + 2 * b], wring, xres, w, lane);
        } else {
            conv_wino<F, false>(ldsb, vbase, zero_off, r1, r2, ta.b[1 + 2 * b], wring, xres, w, lane, trw);
            conv_wino<F, true>(ldsb, vbase, zero_off, r2, r3, ta.b[2 + 2 * b], wring, xres, w, lane);
        }
        if (b < 12) WC_STAMP(3 + b);
    }
#ifdef AZ_WINO_TRACE
    unsigned long long* trh = trc ? trc - 16 * w + 9 : nullptr;   // wave 0's slots 9-11: heads A, C, log slots
#else
    unsigned long long* trh = nullptr;
#endif
    heads_group<F, RSF, 1, NT, SEARCH, true>(ldsb, reinterpret_cast<float*>(V), 0, 1, row0, tid, ta.head_frag32, ta.head,
                                             pol_out, val_out, so, trh);
    WC_STAMP(15);
#undef WC_STAMP
}

// one board (batch row row0) through the Winograd f32 tower, dispatching on F
template <int F, bool SEARCH>
__device__ __forceinline__ void tower32w_board(const float* __restrict__ planes, const TowerArgs& ta, int row0,
                                               float* __restrict__ pol_out, float* __restrict__ val_out,
                                               const SearchOut& so, int tid) {
    if constexpr (F == 256 && AZ_WINO_DT) {
        tower32w_board_dt<SEARCH>(planes, ta, row0, pol_out, val_out, so, tid);
        return;
    } else {
        tower32w_board_shared<F, SEARCH>(planes, ta, row0, pol_out, val_out, so, tid);
    }
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
#ifdef AZ_SIMS_TRACE   // experiment: per-game cycles in the tree phase / the tower phase (tools/sims_trace.py)
    unsigned long long c_tree = 0, c_tower = 0, n_eval = 0, t0 = __builtin_amdgcn_s_memtime(), t1 = t0;
#endif
    for (int step = step0; step <= step1; step++) {
        // indices laundered per simulation so that neither phase's loop-invariant address
        // arithmetic is hoisted across the other (it would stay live through it and spill)
        const int tid = vgpr_index(threadIdx.x), g = vgpr_index(blockIdx.x);
        const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
        if (w == 0) {
            if (step > step0) {                        // the previous simulation's backup
                backup_game(E, g, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
            int kind = X_NONE, nid = -1;
            if (step < step1) {
                select_game(E, g, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                kind = expand_leaf_wave<1>(E, g, lane, &nid, step);   // wave 0 only
                if (lane == 0) {
                    if (kind == X_ROW) {
                        E.row_game[g] = g;
                        E.row_node[g] = nid;
                        E.leaf_row[g] = g;
                        atomicAdd(&E.batch_hist[step], 1);
                        atomicAdd(&E.ctr->evals, 1ull);
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
#ifdef AZ_SIMS_TRACE
        t1 = __builtin_amdgcn_s_memtime();
        c_tree += t1 - t0;
#endif
        if (kind == X_ROW) {
            if constexpr (BF16) tower_board<F, true>(nullptr, ta, g, 1, nullptr, nullptr, so, tid);
            else tower32w_board<F, true>(nullptr, ta, g, nullptr, nullptr, so, tid);
        }
        __syncthreads();
#ifdef AZ_SIMS_TRACE
        t0 = __builtin_amdgcn_s_memtime();
        c_tower += t0 - t1;
        n_eval += kind == X_ROW;
#endif
    }
#ifdef AZ_SIMS_TRACE
    if (threadIdx.x == 0) {
        unsigned long long* tr = E.trace + (size_t)vgpr_index(blockIdx.x) * 16;
        tr[8] += c_tree; tr[9] += c_tower; tr[10] += n_eval; tr[11] += (unsigned long long)(step1 - step0 + 1);
    }
#endif
}

bool tower_supported(const NetDev* n) {
    return (n->dtype == AZ_DTYPE_BF16 || n->dtype == AZ_DTYPE_F32) && n->blocks <= 40 &&
           (n->filters == 256 || n->filters == 128 || n->filters == 64 || n->filters == 32);
}

bool wino_supported(const NetDev* n) {
    return n->dtype == AZ_DTYPE_F32 && n->winograd && n->filters >= 64 && (int)n->wino_w.size() == 2 * n->blocks;
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
    ta.blocks = n->blocks;
    return ta;
}

bool sims_persistent_supported(const NetDev* n) {
#if defined(AZ_TOWER_TRACE) || defined(AZ_WINO_TRACE)
    // trace builds stamp one tower launch into a buffer only tower_forward allocates (the
    // persistent kernel's TowerArgs carry no trace buffer: its stamps would write through null)
    return false;
#endif
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
#if defined(AZ_TOWER_TRACE) || defined(AZ_WINO_TRACE)
#ifndef AZ_TOWER_TRACE
#define AZ_TOWER_TRACE AZ_WINO_TRACE
#endif
    // experiment only: stamp launch number AZ_TOWER_TRACE of this process into $AZ_TOWER_TRACE_FILE
    static unsigned long long* trbuf = nullptr;
    static int launch_no = 0;
    if (!trbuf) (void)hipMalloc(&trbuf, (size_t)(rows + 8) * TR_SLOTS * 8);
    ta.trace = trbuf;
    const bool dump = ++launch_no == AZ_TOWER_TRACE;
#endif
    SearchOut dummy;
    memset(&dummy, 0, sizeof(dummy));
    const SearchOut& s = so ? *so : dummy;
#if defined(AZ_TOWER_TRACE) || defined(AZ_WINO_TRACE)
#define TRACE_DUMP(grid)                                                                                   \
    if (dump) {                                                                                            \
        std::vector<unsigned long long> h((size_t)(grid) * TR_SLOTS);                                      \
        (void)hipStreamSynchronize(st);                                                                    \
        (void)hipMemcpy(h.data(), trbuf, h.size() * 8, hipMemcpyDeviceToHost);                             \
        if (FILE* f = fopen(getenv("AZ_TOWER_TRACE_FILE") ? getenv("AZ_TOWER_TRACE_FILE") : "tower_trace.bin", "wb")) { \
            fwrite(h.data(), 8, h.size(), f);                                                              \
            fclose(f);                                                                                     \
        }                                                                                                  \
    }
#else
#define TRACE_DUMP(grid)
#endif
#define AZ_TOWER(FF)                                                                                           \
    if (n->filters == FF) {                                                                                    \
        constexpr int BPB = TowerCfg<FF>::BPB;                                                                 \
        constexpr int NT = (FF / (16 * TowerCfg<FF>::NCO)) * TowerCfg<FF>::WB * 64;                            \
        const int grid = (rows + BPB - 1) / BPB;                                                               \
        if (so) tower_kernel<FF, true><<<grid, NT, 0, st>>>((const __bf16*)planes, ta, count, rows, pol, val, s); \
        else tower_kernel<FF, false><<<grid, NT, 0, st>>>((const __bf16*)planes, ta, count, rows, pol, val, s);  \
        TRACE_DUMP(grid);                                                                                      \
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
            TRACE_DUMP(rows);                                                                                  \
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

// wino.h -- the f32 Winograd F(2x2, 3x3) conv of one board, shared by the inference tower
// (tower.hip: tower32w_kernel, k_sims32w) and the training step (train.hip: conv_wino_train_kernel).
#pragma once
#include "az_internal.h"

namespace azi {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

// Packed f32 adds (v_pk_add_f32 / v_pk_fma_f32: two results per VALU issue) with the per-half source
// selects and negations written out.  Left to itself the compiler packed the transforms' adds but
// moved operands into register pairs first (one v_mov per packed add), and VALU issue is what the
// f32 MFMA pipe does not hide.  No memory operands: the waits stay the compiler's.
#define AZ_PK2(name, mods)                                                                    \
    __device__ __forceinline__ f32x2 name(f32x2 a, f32x2 b) {                                 \
        f32x2 r;                                                                              \
        asm("v_pk_add_f32 %0, %1, %2 " mods : "=v"(r) : "v"(a), "v"(b));                      \
        return r;                                                                             \
    }
#define AZ_PK3(name, mods)                                                                    \
    __device__ __forceinline__ f32x2 name(f32x2 a, f32x2 m, f32x2 b) {                        \
        f32x2 r;                                                                              \
        asm("v_pk_fma_f32 %0, %1, %2, %3 " mods : "=v"(r) : "v"(a), "v"(m), "v"(b));          \
        return r;                                                                             \
    }
AZ_PK2(pk_add, "")                                             // (a.x + b.x, a.y + b.y)
AZ_PK2(pk_sub, "neg_lo:[0,1] neg_hi:[0,1]")                    // (a.x - b.x, a.y - b.y)
AZ_PK2(pk_rowa, "op_sel_hi:[1,0] neg_lo:[0,1]")                // (a.x - b.x, a.y + b.x)
AZ_PK2(pk_rowb, "op_sel:[1,0] neg_lo:[0,1] neg_hi:[0,1]")      // (a.y - b.x, a.y - b.y)
AZ_PK2(pk_negx_add, "neg_lo:[1,1]")                            // (-a.x - b.x, a.y + b.y)
AZ_PK2(pk_negx_sub, "neg_lo:[1,0] neg_hi:[0,1]")               // (-a.x + b.x, a.y - b.y)
AZ_PK3(pk_fma_m0_sub, "op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]")    // (a.x m.x - b.x, a.y m.x - b.y)
AZ_PK3(pk_sub_m3, "op_sel:[0,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]")          // (b.x - a.x m.y, b.y - a.y m.y)
AZ_PK3(pk_negx_fma_m0, "op_sel_hi:[1,0,1] neg_lo:[1,0,0] neg_hi:[0,0,1]")   // (-a.x m.x + b.x, a.y m.x - b.y)
AZ_PK3(pk_negx_sub_m3, "op_sel:[0,1,0] neg_lo:[0,0,1] neg_hi:[1,0,0]")      // (a.x m.y - b.x, -a.y m.y + b.y)

// Phase stamps for the tower trace build (make EXTRA=-DAZ_TOWER_TRACE, tools/tower_trace.c): shader
// clock of one wave at a phase boundary, written by lane 0 through a vector store; `tr` is
// nullptr (no code) in every other build
__device__ __forceinline__ void wino_stamp(unsigned long long* tr, int k) {
#ifdef AZ_TOWER_TRACE
    if (tr) {
        __builtin_amdgcn_sched_barrier(0);
        unsigned long long t;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        if ((threadIdx.x & 63) == 0) tr[k] = t;
    }
#else
    (void)tr; (void)k;
#endif
}

// zero squares before and after ACT ([64 squares][F/4 + 2 slots]): the transform reads the rows
// above / below the board there
constexpr int WINO_PAD_SQ = 8;

// ====================================================================== f32 Winograd tower
// tower32w_kernel: the same f32 tower with every residual 3x3 conv as Winograd F(2x2, 3x3)
// (Lavin & Gray): the 8x8 board is 16 output tiles of 2x2 whose 4x4 input patches are
// transformed V = B^T d B (16 points xi), the weights were transformed on the host
// U = G g G^T (f64, rounded once to f32), M[xi] = U[xi] V[xi] summed over the input channels is
// 16 GEMMs of F x 16 tiles x F on v_mfma_f32_16x16x4_f32 (exact f32 products), and
// Y = A^T M A.  2.25x fewer MFMAs than the direct conv (16 tiles x 16 points vs 64 squares x 9
// taps).  Numerics: f32 throughout; the transforms' rounding adds ~1.3x the direct f32 error
// (numpy check), checked against the oracle within the f32 tolerance.
// One board per workgroup:
//   ACT [64 squares][F/4 + 2 slots] f32 in LDS -- the layer input, overwritten in place by the
//       output (the block input x stays in the registers of the wave that owns it, as the residual),
//       with WINO_PAD_SQ zero squares before and after it;
//   V   [16 xi][channel quads][16 tiles][4] f32 in CH-channel chunks (double-buffered when the
//       input takes more than one chunk): chunk c+1 is transformed by all waves, one (channel,
//       tile) item per thread, while the MFMAs of chunk c run; one barrier per chunk;
//   weights [F/16 ci groups][16 xi][F/16 co groups][64 lanes][4] f32 per conv, streamed from L2
//       through a register ring of PF steps that carries across layers.
// Step constants (C3 / C2 A/B logs: profiles/r02_ab_wino_s9_knobs_c3.log, r02_ab_wino64_*):
//   WINO_TSPLIT 2  steps between a chunk's patch reads and their transform + V writes (8 -> 2: -2 %)
//   WINO_TSTAG 16  steps by which the second wave of each SIMD pair delays its transform (-0.4 %)
//   WINO_LA 4      B fragments read ahead from V
constexpr int WINO_TSPLIT = 2, WINO_TSTAG = 16, WINO_LA = 4;
// timing-only knob (wrong results): -DAZ_WINO_WFAKE=1 makes every ring step re-read the first two
// steps' weights (L2 / L1 hits), to price the weight stream from L2
#if defined(AZ_WINO_WFAKE) && AZ_WINO_WFAKE
#define WINO_WSTEP(t) ((t) & 1)
#else
#define WINO_WSTEP(t) (t)
#endif

// Per filter count: NWV waves per workgroup, NN 16-channel output fragments per wave, XS points
// per ring step, CH input channels per transform chunk (V buffer = CH KB), PF ring steps of
// weight prefetch.  Every wave owns NN output fragments x all 16 points.
//   F = 256: 8 waves (two per SIMD) x 32 output channels, one point per step (two independent
//            accumulator chains per step), 32-channel chunks;
//   F = 128: 8 waves x 16 channels, two points per step (still two chains: the f32 MFMA's
//            dependent latency exceeds its issue interval);
//   F = 64:  4 waves (one per SIMD) x 16 channels, two points per step, the whole 64-channel input
//            transformed as one chunk (one transform phase and one barrier per conv: C2 A/B -8 %).
template <int F> struct WinoCfg;
template <> struct WinoCfg<256> { static constexpr int NWV = 8, NN = 2, XS = 1, CH = 32, PF = 2; };
template <> struct WinoCfg<128> { static constexpr int NWV = 8, NN = 1, XS = 2, CH = 32, PF = 2; };
template <> struct WinoCfg<64> { static constexpr int NWV = 4, NN = 1, XS = 2, CH = 64, PF = 2; };
// Winograd weight fragment offsets: wave w's lane base (output fragments NN w..) and the byte
// offset of ring step t (16-channel group kl = t / 16, point t % 16) of chunk cg
template <int F> __device__ __forceinline__ int wino_voff(int w, int lane) {
    return (WinoCfg<F>::NN * w * 64 + lane) * 16;
}
template <int F> __device__ __forceinline__ int wino_toff(int cg, int t) {
    constexpr int KPC = WinoCfg<F>::CH / 16, CF = F / 16;
    return ((cg * KPC + t / 16) * 16 + t % 16) * CF * 1024;
}

// The input transform V[buf] <- B^T d B of one chunk, one (channel, tile) item per thread and
// item slot.  Items: wave w covers tile row ty = w & 3 and 16 channels per item: channel
// 16 (w >> 2 + g + it NWV / 4) + (lane & 15) of the chunk, tile (w & 3, lane >> 4) -- a patch read
// then touches 4 tiles of one row x 16 consecutive channels: conflict-free with the ACT row stride
// of 8 banks mod 64.  g = 1 names the item of the wave NWV / 4 waves later (used when one wave
// transforms for two).  In two halves: load issues the patch reads, store transforms and writes V.
// d[it][j] = patch column j as row pairs {rows 0, 1}, {rows 2, 3} (one ds_read2st64_b32 each).
// Element (i, j) of a patch is square (2 ty - 1 + i, 2 tl - 1 + j): rows off the board fall in the
// zero squares before / after ACT (WINO_PAD_SQ), so every row offset is an instruction immediate;
// the off-board columns (tl = 0: j = 0, tl = 3: j = 3) are read at a clamped on-board column (3 / 4:
// keeps the 32-lane groups of each read on distinct banks) and multiplied by 0 in store.
template <int F> struct WinoXf {
    static constexpr int NWV = WinoCfg<F>::NWV, CH = WinoCfg<F>::CH, RS = F / 4 + 2;
    static constexpr int VBYTES = CH * 1024, XST = CH * 64, IT = CH * 16 / (NWV * 64);
    static constexpr int R16 = RS * 16, ROW = 8 * R16;
    typedef f32x2 Patch[IT][4][2];
    char* ldsb;
    int vbase, w, lane, tty, ttx;
    __device__ __forceinline__ WinoXf(char* l, int vb, int w_, int lane_)
        : ldsb(l), vbase(vb), w(w_), lane(lane_), tty(w_ & 3), ttx(lane_ >> 4) {}
    __device__ __forceinline__ int tchan(int it, int g) const { return 16 * ((w >> 2) + g + it * (NWV / 4)) + (lane & 15); }
    __device__ __forceinline__ int vwr(int tch) const {   // + xi * XST
        return (tch >> 2) * 256 + (((4 * tty + ttx) ^ (2 * ((tch >> 2) & 3))) * 16) + (tch & 3) * 4;
    }
    __device__ __forceinline__ void load(int c, Patch& d, int g = 0) const {
        // recomputed per chunk from a laundered index: one loop-invariant register more spilled
        const int tl = vgpr_index(ttx);
        const int pc1 = tl * (2 * R16) + (lane & 15) * 4;
        const int pd0 = tl > 0 ? -R16 : 3 * R16, pd3 = tl < 3 ? 2 * R16 : -2 * R16;
#pragma unroll
        for (int it = 0; it < IT; it++) {
            // tchan(it) - (lane & 15) is wave-uniform
            const int b1 = pc1 + (2 * tty - 1) * ROW + (c * CH + tchan(it, g) - (lane & 15)) * 4;
            const int cb[4] = {b1 + pd0, b1, b1 + R16, b1 + pd3};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const char* p = ldsb + cb[j];
                d[it][j][0] = f32x2{*reinterpret_cast<const float*>(p), *reinterpret_cast<const float*>(p + ROW)};
                d[it][j][1] = f32x2{*reinterpret_cast<const float*>(p + 2 * ROW), *reinterpret_cast<const float*>(p + 3 * ROW)};
            }
        }
    }
    // B^T d B of one channel's patch: d[j] = column j as row pairs {rows 0, 1}, {rows 2, 3};
    // v[k][rp] = (points (2 rp) 4 + k, (2 rp + 1) 4 + k); m = (m0, m3): 0 where patch column 0 / 3
    // is off the board
    static __device__ __forceinline__ void xform(const f32x2 (&d)[4][2], f32x2 m, f32x2 (&v)[4][2]) {
        // rows: A[j] = (tt0, tt1) = (e0 - e2, e1 + e2), B[j] = (-tt2, tt3) = (e1 - e2, e1 - e3)
        f32x2 A[4], B[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            A[j] = pk_rowa(d[j][0], d[j][1]);
            B[j] = pk_rowb(d[j][0], d[j][1]);
        }
        // columns, two rows at a time: v0 = t0 m0 - t2, v1 = t1 + t2, v2 = t2 - t1, v3 = t1 - t3 m3
        // (the same roundings as the scalar form: every multiply is by 1 or 0)
        v[0][0] = pk_fma_m0_sub(A[0], m, A[2]);
        v[1][0] = pk_add(A[1], A[2]);
        v[2][0] = pk_sub(A[2], A[1]);
        v[3][0] = pk_sub_m3(A[3], m, A[1]);
        v[0][1] = pk_negx_fma_m0(B[0], m, B[2]);
        v[1][1] = pk_negx_add(B[1], B[2]);
        v[2][1] = pk_negx_sub(B[2], B[1]);
        v[3][1] = pk_negx_sub_m3(B[3], m, B[1]);
    }
    __device__ __forceinline__ void store(int buf, const Patch& d, int g = 0) const {
        const int tl = vgpr_index(ttx);
        const f32x2 m = f32x2{tl > 0 ? 1.0f : 0.0f, tl < 3 ? 1.0f : 0.0f};
#pragma unroll
        for (int it = 0; it < IT; it++) {
            f32x2 v[4][2];   // [column k][row pair]
            xform(d[it], m, v);
            char* vb = ldsb + vbase + buf * VBYTES + vwr(tchan(it, g));
#pragma unroll
            for (int k = 0; k < 4; k++)
#pragma unroll
                for (int rp = 0; rp < 2; rp++) {
                    *reinterpret_cast<float*>(vb + ((2 * rp) * 4 + k) * XST) = v[k][rp].x;
                    *reinterpret_cast<float*>(vb + ((2 * rp + 1) * 4 + k) * XST) = v[k][rp].y;
                }
        }
    }
    // the first NWV / 2 waves transform chunk c into V[buf] for all NWV waves (their own items and
    // those of the waves NWV / 2 later): F = 256 only (IT = 1, NWV = 8)
    __device__ __forceinline__ void both(int c, int buf) const {
        static_assert(IT == 1 && NWV == 8, "two items per thread of the first half");
        Patch d0, d1;
        load(c, d0, 0);
        load(c, d1, 1);
        store(buf, d0, 0);
        store(buf, d1, 1);
    }
};

// DPP row shift within the 16-lane rows: lane l reads lane l - N (SHR) / l + N (SHL); a source
// outside the row reads 0 (bound_ctrl)
template <int CTRL> __device__ __forceinline__ float row_dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
constexpr int DPP_SHL = 0x100, DPP_SHR = 0x110;

// The next conv's input transform straight from a wave's conv outputs (F = 64: each wave's 16
// output channels x all 16 tiles are one quarter of the single 64-channel chunk).  o[q] = the
// lane's 4 channels (quad h of the wave's 16) at square (2 ty + q / 2, 2 tx + q % 2) of tile
// l16 = 4 ty + tx.  A tile's 4x4 patch reaches one square into each neighbouring tile; the
// neighbours' values come over DPP row shifts (tile +-1 = lane +-1, +-4 = lane +-4 within the
// 16-lane row): off-board rows read 0 (outside the row), off-board columns read a finite value
// that the transform multiplies by 0 -- exactly WinoXf::load + store on the same outputs in LDS,
// bit for bit.  Writes the 16 points x 4 channels of the lane's (quad, tile) into V at vdst with
// one ds_write_b128 per point.
AZ_PK2(pkc_nadd, "neg_lo:[1,1] neg_hi:[1,1]")                 // (-a.x - b.x, -a.y - b.y)
AZ_PK3(pkc_fma_nc, "neg_lo:[0,0,1] neg_hi:[0,0,1]")            // (a.x m.x - c.x, a.y m.y - c.y)
AZ_PK3(pkc_nfma, "neg_lo:[1,0,0] neg_hi:[1,0,0]")              // (-a.x m.x + c.x, -a.y m.y + c.y)
#undef AZ_PK2
#undef AZ_PK3
template <int F>
__device__ __forceinline__ void wino_xform_regs(const f32x4 (&o)[4], char* __restrict__ vdst, int w, int lane) {
    static_assert(F == 64 && WinoCfg<F>::NN == 1, "one chunk, one output fragment per wave");
    constexpr int XST = WinoCfg<F>::CH * 64;
    const int l16 = lane & 15, h = lane >> 4, tx = l16 & 3;
    const int cq = w * 4 + h;                                       // channel quad of the chunk
    const float m0 = tx > 0 ? 1.0f : 0.0f, m3 = tx < 3 ? 1.0f : 0.0f;
    const f32x2 m0v = f32x2{m0, m0}, m3v = f32x2{m3, m3};
    f32x4 out[16];
#pragma unroll
    for (int cp = 0; cp < 2; cp++) {   // channel pairs (2 cp, 2 cp + 1), packed in one f32x2
        auto own = [&](int q) { return cp ? f32x2{o[q][2], o[q][3]} : f32x2{o[q][0], o[q][1]}; };
        auto nb = [&](auto dpp, int q) { const f32x2 v = own(q); return f32x2{dpp(v.x), dpp(v.y)}; };
        auto shr1 = [](float x) { return row_dpp<DPP_SHR + 1>(x); };
        auto shr3 = [](float x) { return row_dpp<DPP_SHR + 3>(x); };
        auto shr4 = [](float x) { return row_dpp<DPP_SHR + 4>(x); };
        auto shr5 = [](float x) { return row_dpp<DPP_SHR + 5>(x); };
        auto shl1 = [](float x) { return row_dpp<DPP_SHL + 1>(x); };
        auto shl3 = [](float x) { return row_dpp<DPP_SHL + 3>(x); };
        auto shl4 = [](float x) { return row_dpp<DPP_SHL + 4>(x); };
        auto shl5 = [](float x) { return row_dpp<DPP_SHL + 5>(x); };
        // P[i][j]: patch rows i (square row 2 ty - 1 + i), columns j
        const f32x2 P[4][4] = {
            {nb(shr5, 3), nb(shr4, 2), nb(shr4, 3), nb(shr3, 2)},
            {nb(shr1, 1), own(0), own(1), nb(shl1, 0)},
            {nb(shr1, 3), own(2), own(3), nb(shl1, 2)},
            {nb(shl3, 1), nb(shl4, 0), nb(shl4, 1), nb(shl5, 0)}};
        // rows (as WinoXf::xform): R0 = P0 - P2, R1 = P1 + P2, nR2 = P1 - P2, R3 = P1 - P3
        f32x2 R[4][4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            R[0][j] = pk_sub(P[0][j], P[2][j]);
            R[1][j] = pk_add(P[1][j], P[2][j]);
            R[2][j] = pk_sub(P[1][j], P[2][j]);
            R[3][j] = pk_sub(P[1][j], P[3][j]);
        }
        // columns: the operations of WinoXf::xform per point, two channels per instruction
        f32x2 V[4][4];
        V[0][0] = pkc_fma_nc(R[0][0], m0v, R[0][2]);
        V[0][1] = pk_add(R[0][1], R[0][2]);
        V[0][2] = pk_sub(R[0][2], R[0][1]);
        V[0][3] = pkc_nfma(R[0][3], m3v, R[0][1]);
        V[1][0] = pkc_fma_nc(R[1][0], m0v, R[1][2]);
        V[1][1] = pk_add(R[1][1], R[1][2]);
        V[1][2] = pk_sub(R[1][2], R[1][1]);
        V[1][3] = pkc_nfma(R[1][3], m3v, R[1][1]);
        V[2][0] = pkc_nfma(R[2][0], m0v, R[2][2]);
        V[2][1] = pkc_nadd(R[2][1], R[2][2]);
        V[2][2] = pk_sub(R[2][1], R[2][2]);
        V[2][3] = pkc_fma_nc(R[2][3], m3v, R[2][1]);
        V[3][0] = pkc_fma_nc(R[3][0], m0v, R[3][2]);
        V[3][1] = pk_add(R[3][1], R[3][2]);
        V[3][2] = pk_sub(R[3][2], R[3][1]);
        V[3][3] = pkc_nfma(R[3][3], m3v, R[3][1]);
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) {
                out[4 * a + b][2 * cp] = V[a][b].x;
                out[4 * a + b][2 * cp + 1] = V[a][b].y;
            }
    }
    char* vb = vdst + cq * 256 + ((l16 ^ (2 * (cq & 3))) * 16);
#pragma unroll
    for (int p = 0; p < 16; p++) *reinterpret_cast<f32x4*>(vb + p * XST) = out[p];
}

// wino_core: one Winograd conv of the board whose layer input is in ACT ([64 squares][F/4 + 2
// slots] f32 at ldsb, WINO_PAD_SQ zero squares on either side), V buffers at vbase: every wave's y[n][q] = this wave's outputs (output
// fragment n, tile lane & 15, square (2 ty + q / 2, 2 tx + q % 2), channels co0 + 16 n + 0..3)
// + bias (nullptr: none).  Ends without a workgroup barrier: other waves may still be issuing
// MFMAs on the last V buffer, but every read of ACT and of the other V buffer is done, so the caller
// may overwrite ACT; it must pass a barrier before the next wino_core (which writes V) or before
// reusing V.
// wr: the weight ring; holds this conv's first PF steps on entry and the next conv's (rN) on
// exit, so no layer starts on a cold weight fetch
template <int F>
__device__ __forceinline__ void wino_core(char* __restrict__ ldsb, int vbase,
                                          const __amdgpu_buffer_rsrc_t rW, const __amdgpu_buffer_rsrc_t rN,
                                          const float* __restrict__ bias,
                                          f32x4 (&wr)[WinoCfg<F>::PF][WinoCfg<F>::XS][WinoCfg<F>::NN], int w,
                                          int lane, f32x4 (&y)[WinoCfg<F>::NN][4], bool pre = false,
                                          unsigned long long* tr = nullptr) {
    constexpr int CF = F / 16;
    constexpr int NWV = WinoCfg<F>::NWV, NN = WinoCfg<F>::NN, XS = WinoCfg<F>::XS;
    constexpr int CH = WinoCfg<F>::CH, VBYTES = CH * 1024, XST = CH * 64;   // V buffer, xi stride
    constexpr int IT = CH * 16 / (NWV * 64);                       // transform items per thread per chunk
    // t = (16-channel group kl, point t % 16) pairs of this wave per chunk; a ring step covers XS
    constexpr int NCHUNK = F / CH, KPC = CH / 16, SPC = KPC * 16, SPX = SPC / XS;
    constexpr int PF = WinoCfg<F>::PF, LA = WINO_LA * XS;
    static_assert(NN * 16 * NWV == F && IT * NWV * 64 == CH * 16 && NWV % 4 == 0 && IT >= 1, "Winograd config");
    static_assert(SPX % PF == 0 && SPC % LA == 0 && 16 % XS == 0, "ring slots must be compile-time");
    const int l16 = lane & 15, h = lane >> 4;
    // V[xi][quad cq][tile slot][4]: tile slot = tile ^ 2 (cq & 3).  gfx950 services a ds_read_b128
    // in the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): each group holds quads h and
    // h + 1 of a fragment at complementary tile sets, and the XOR by 2h keeps their 16 slots distinct
    // (64 banks); a ds_write_b32 of the transform (32-lane groups, 32 banks) then covers 8 distinct
    // slot values mod 8, so both are conflict-free (an XOR by 4h, laid out for groups of 16
    // consecutive lanes, made every B-fragment read 2-way: PMC 48 % of LDS cycles were conflicts)
    const int vrd = h * 256 + ((l16 ^ (2 * h)) * 16);               // + xi * XST + k * 1024 (cq = 4k + h, cq & 3 = h)
    const WinoXf<F> xf(ldsb, vbase, w, lane);
    const int co0 = w * 16 * NN + h * 4;
    // (peeling the first chunk so that its MFMAs take C = 0 instead of this zeroing pass made the
    // register allocation spill: 30 VGPRs at F = 256)
    f32x4 acc[16][NN];
#pragma unroll
    for (int x = 0; x < 16; x++)
#pragma unroll
        for (int n = 0; n < NN; n++) {
            if constexpr (F == 256) {   // accumulators in VGPRs: 64-bit moves (the compiler's zeroing was 128 32-bit moves)
                f32x2 z0, z1;
                asm volatile("v_mov_b64 %0, 0" : "=v"(z0));
                asm volatile("v_mov_b64 %0, 0" : "=v"(z1));
                acc[x][n] = f32x4{z0.x, z0.y, z1.x, z1.y};
            } else {                    // F = 64 keeps them in AGPRs, zeroed there directly
                acc[x][n] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    // weight ring: fragment (16-channel group kc, point xi, co/16 = NN w + n) at ((kc 16 + xi) CF + co/16) KB
    const int voff = wino_voff<F>(w, lane);
    if (!pre) {   // chunk 0 not transformed by the caller
        f32x2 d0[IT][4][2];
        xf.load(0, d0);
        xf.store(0, d0);
        __syncthreads();
    }
    wino_stamp(tr, 1);
    // B fragment of this wave's step t: 16-channel group t / 16 of the chunk, point t % 16
    auto boff = [](int t) { return (t / 16) * 1024 + (t % 16) * XST; };
#pragma unroll 1
    for (int c = 0; c < NCHUNK; c++) {
        f32x2 dn[IT][4][2];
        const int vb = vbase + (c & 1) * VBYTES + vrd;
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
                if (t + LA < SPC) bq[t % LA] = *reinterpret_cast<const f32x4*>(ldsb + vb + boff(t + LA));
            }
            f32x4 a[XS][NN];
#pragma unroll
            for (int xs = 0; xs < XS; xs++)
#pragma unroll
                for (int n = 0; n < NN; n++) a[xs][n] = wr[st % PF][xs][n];
            {
                // ring step st + PF: the steps of a conv are linear in the weights; past this
                // conv's last step the refills read the next conv's first steps
                const int cadd = (st + PF) / SPX;
                const bool nxt = cadd > 0 && !more;
                const int tn = c * SPX + st + PF;
                const int to = (nxt ? tn - NCHUNK * SPX : tn) * XS;
                // the step's (wave-uniform) offset rides in the instruction's SGPR offset, the
                // fragment's in the lane offset + immediate: no VALU address arithmetic per load
#pragma unroll
                for (int xs = 0; xs < XS; xs++)
#pragma unroll
                    for (int n = 0; n < NN; n++)
                        wr[st % PF][xs][n] = __builtin_bit_cast(
                            f32x4, __builtin_amdgcn_raw_buffer_load_b128(nxt ? rN : rW, voff + n * 1024,
                                                                         WINO_WSTEP(to + xs) * CF * 1024, 0));
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int xs = 0; xs < XS; xs++)
#pragma unroll
                    for (int n = 0; n < NN; n++) {
                        const int x = (st * XS + xs) % 16;
                        acc[x][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[xs][n][s4], B[xs][s4], acc[x][n], 0, 0, 0);
                    }
            __builtin_amdgcn_sched_barrier(0);
            // the next chunk's transform.  F = 256: the first wave of each SIMD pair, which runs ahead
            // of its partner by ~30 % of a chunk, transforms both waves' items after
            // its last step, beside its partner's last MFMAs (C3 A/B: tower -1.1 % against one item
            // per wave at staggered steps); other F: one item per wave, the two waves of a SIMD pair
            // WINO_TSTAG steps apart (a stagger that would not fit in this F's chunk is dropped)
            if (st == 4) wino_stamp(tr, 20 + c);
            if constexpr (F == 256) {
                (void)dn;
                if (st == SPX - 1 && more && w < NWV / 2) xf.both(c + 1, (c + 1) & 1);
            } else {
                constexpr int TSG = (WINO_TSTAG + WINO_TSPLIT) / XS < SPX ? WINO_TSTAG : 0;
                const bool late = TSG > 0 && w >= NWV / 2;
                if (st == 0 && more && !late) xf.load(c + 1, dn);
                if (TSG > 0 && st == TSG / XS && more && late) xf.load(c + 1, dn);
                if (st == WINO_TSPLIT / XS && more && !late) xf.store((c + 1) & 1, dn);
                if (TSG > 0 && st == (TSG + WINO_TSPLIT) / XS && more && late) xf.store((c + 1) & 1, dn);
            }
        }
        wino_stamp(tr, 12 + c);
        // no barrier after the last chunk: the last transform reads of ACT and writes of V were
        // ordered by the previous chunk's barrier, so the waves that finish first start their
        // output transform beside the others' last MFMAs (C3 A/B: tower -0.6 %)
        if (more) __syncthreads();
        wino_stamp(tr, 2 + c);
    }
    // output transform Y = A^T M A per (output fragment n, channel pair), + bias: the two channels
    // of a pair sit in consecutive accumulator registers, so every add is one v_pk_add_f32
#pragma unroll
    for (int n = 0; n < NN; n++) {
        const f32x4 bb = bias ? *reinterpret_cast<const f32x4*>(bias + co0 + n * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 2; p++) {
            f32x2 m[16];
#pragma unroll
            for (int x = 0; x < 16; x++) m[x] = p ? f32x2{acc[x][n][2], acc[x][n][3]} : f32x2{acc[x][n][0], acc[x][n][1]};
            const f32x2 br = p ? f32x2{bb[2], bb[3]} : f32x2{bb[0], bb[1]};
            f32x2 s0[4], s1[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                s0[j] = pk_add(pk_add(m[j], m[4 + j]), m[8 + j]);
                s1[j] = pk_sub(pk_sub(m[4 + j], m[8 + j]), m[12 + j]);
            }
            const f32x2 q0 = pk_add(pk_add(pk_add(s0[0], s0[1]), s0[2]), br);
            const f32x2 q1 = pk_add(pk_sub(pk_sub(s0[1], s0[2]), s0[3]), br);
            const f32x2 q2 = pk_add(pk_add(pk_add(s1[0], s1[1]), s1[2]), br);
            const f32x2 q3 = pk_add(pk_sub(pk_sub(s1[1], s1[2]), s1[3]), br);
            y[n][0][2 * p] = q0.x; y[n][0][2 * p + 1] = q0.y;
            y[n][1][2 * p] = q1.x; y[n][1][2 * p + 1] = q1.y;
            y[n][2][2 * p] = q2.x; y[n][2][2 * p + 1] = q2.y;
            y[n][3][2 * p] = q3.x; y[n][3][2 * p + 1] = q3.y;
        }
    }
}

}  // namespace azi

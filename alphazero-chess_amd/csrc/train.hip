// train.hip -- the training step of training.rs:137-200 / 277-292 on gfx950, f32 end to end
// (the reference trains in f32: burn 0.18 CUDA backend, FullPrecisionSettings records).
//
// Activations are NHWC f32 [row = board*64 + square][channels].  Every convolution is an
// implicit GEMM on v_mfma_f32_16x16x4_f32 (exact f32 FMA chains -- the reference's precision):
//   forward      Y[r][n]      = b[n] + sum_t sum_k X[r + d_t][k] * Wf[t][k][n]
//   data grad    dX[r][k]     =        sum_t sum_n dY[r + d_t][n] * Wd[t][n][k],  Wd[t] = Wf[8-t]^T
//   weight grad  dWf[t][k][n] = sum_r X[r + d_t][k] * dY[r][n]    (row splits, fixed-order reduce)
// where d_t is the 3x3 tap shift inside the 8x8 board with zero padding (agent.rs:21-23,
// PaddingConfig2d::Same); the 1x1 head convs and the Linear layers are the TAPS = 1 case over
// generic rows.  BatchNorm runs in training mode (batch statistics, biased variance, running
// statistics updated with momentum 0.1 -- burn BatchNorm::forward_train, restated), then ReLU /
// residual; the loss is training.rs:277-292 (policy CE with log(p + 1e-5), 0.5 * MSE value);
// gradients are clipped by value to [-1, 1] and applied with burn's AdamW (training.rs:63-66:
// beta 0.9 / 0.999, eps 1e-5 outside the sqrt, decoupled weight decay 1e-4).
// Every reduction has a fixed order, so a step is bit-reproducible run to run.
// At F = 256 the residual convs run as Winograd F(2x2,3x3) (wino.h), each BatchNorm's apply staged
// in the next conv and its backward in the next data-grad conv (tr::BnIn / tr::BnBack).
// Data-parallel (training.rs:137-190 on N GPUs): the flat gradient is summed over
// ranks with ncclAllReduce (RCCL over xGMI) on the trainer's stream before clipping.  Per-rank
// batches (default): BatchNorm running statistics are averaged the same way after the step.
// Sharded batch (az_trainer_set_sharded): the ranks' batches are one batch, every BatchNorm's
// statistics and backward sums are exchanged inside the step (bn_local / bn_global kernels).
#include <math.h>
#include <string.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <initializer_list>
#include <string>
#include <utility>
#include <vector>

#include "az_internal.h"
#include "wino.h"

namespace azi {
namespace tr {

typedef __attribute__((ext_vector_type(4))) float f32x4;

// source row of tap t for row r (board-major rows); false = zero padding
__device__ __forceinline__ bool tap_src(int r, int t, int& src) {
    const int sq = r & 63, rr = (sq >> 3) + t / 3 - 1, ff = (sq & 7) + t % 3 - 1;
    src = (r & ~63) + rr * 8 + ff;
    return (unsigned)rr < 8u && (unsigned)ff < 8u;
}

// ------------------------------------------------------------------ forward / data-grad GEMM
// Tile: 128 rows x 64 columns per 256-thread workgroup (4 waves, 2 x 2: 64 rows x 32 columns per
// wave = 4 x 2 accumulators of 16x16), K staged 16 channels at a time (all TAPS weight slices of
// the chunk in LDS).  Requires K % 16 == 0, N % 16 == 0, ldx/ldy % 4 == 0, and R % 64 == 0 when
// TAPS == 9 (whole boards).
constexpr int CM = 128, CN = 64, CK = 16;
constexpr int XS = CK + 1;     // A-tile row stride (floats): 16 consecutive rows hit 16 banks
constexpr int WS = CN + 16;    // B-tile row stride: rows k and k+1 land on disjoint bank halves

template <int TAPS>
__global__ void __launch_bounds__(256)
conv_f32_kernel(const float* __restrict__ X, int ldx, int K, const float* __restrict__ W, int N,
                const float* __restrict__ bias, const float* __restrict__ addend, float* __restrict__ Y, int ldy,
                int R) {
    __shared__ float xs[CM * XS + XS];    // + one zero row read by off-board taps
    __shared__ __attribute__((aligned(16))) float ws[TAPS * CK * WS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w & 1, wn = w >> 1;
    const int r0 = blockIdx.x * CM, n0 = blockIdx.y * CN;
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i][0] = acc[i][1] = f32x4{0, 0, 0, 0};
    if (tid < XS) xs[CM * XS + tid] = 0.0f;
    // the next K chunk's X and W slices are read into registers while the current chunk's MFMAs
    // run (software pipeline), then written to LDS after the barrier
    constexpr int NXV = CM * (CK / 4) / 256, NWV = (TAPS * CK * (CN / 4) + 255) / 256;
    float4 xv[NXV], wv[NWV];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int j = 0; j < NXV; j++) {
            const int i = tid + j * 256, rr = i >> 2, c4 = (i & 3) * 4;
            xv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r0 + rr < R) xv[j] = *reinterpret_cast<const float4*>(X + (size_t)(r0 + rr) * ldx + k0 + c4);
        }
#pragma unroll
        for (int j = 0; j < NWV; j++) {
            const int i = tid + j * 256;
            const int t = i / (CK * CN / 4), rem = i % (CK * CN / 4), kk = rem / (CN / 4), n4 = (rem % (CN / 4)) * 4;
            wv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < TAPS * CK * (CN / 4) && n0 + n4 < N)
                wv[j] = *reinterpret_cast<const float4*>(W + ((size_t)t * K + k0 + kk) * N + n0 + n4);
        }
    };
    fetch(0);
    for (int k0 = 0; k0 < K; k0 += CK) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NXV; j++) {
            const int i = tid + j * 256, rr = i >> 2, c4 = (i & 3) * 4;
            float* d = xs + rr * XS + c4;
            d[0] = xv[j].x; d[1] = xv[j].y; d[2] = xv[j].z; d[3] = xv[j].w;
        }
#pragma unroll
        for (int j = 0; j < NWV; j++) {
            const int i = tid + j * 256;
            const int t = i / (CK * CN / 4), rem = i % (CK * CN / 4), kk = rem / (CN / 4), n4 = (rem % (CN / 4)) * 4;
            if (i < TAPS * CK * (CN / 4)) *reinterpret_cast<float4*>(ws + (t * CK + kk) * WS + n4) = wv[j];
        }
        __syncthreads();
        if (k0 + CK < K) fetch(k0 + CK);
#pragma unroll 1
        for (int t = 0; t < TAPS; t++) {
            int aoff[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int row = wm * 64 + i * 16 + (lane & 15);
                if constexpr (TAPS == 9) {
                    int src;
                    const bool ok = tap_src(r0 + row, t, src);
                    aoff[i] = ok ? (src - r0) * XS : CM * XS;
                } else {
                    aoff[i] = row * XS;
                }
            }
#pragma unroll
            for (int kk4 = 0; kk4 < CK / 4; kk4++) {
                const int kq = kk4 * 4 + (lane >> 4);
                float a[4], b[2];
#pragma unroll
                for (int i = 0; i < 4; i++) a[i] = xs[aoff[i] + kq];
#pragma unroll
                for (int j = 0; j < 2; j++) b[j] = ws[(t * CK + kq) * WS + wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int col = n0 + wn * 32 + j * 16 + (lane & 15);
        if (col >= N) continue;
        const float bc = bias ? bias[col] : 0.0f;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int row = r0 + wm * 64 + i * 16 + (lane >> 4) * 4 + g;
                if (row >= R) continue;
                float v = acc[i][j][g];
                if (bias) v += bc;
                if (addend) v += addend[(size_t)row * ldy + col];
                Y[(size_t)row * ldy + col] = v;
            }
    }
}

// ------------------------------------------------------------------ weight-grad GEMM
// Tile: 64 k x 64 n, all TAPS, rows consumed 64 at a time (one board when TAPS == 9) inside the
// workgroup's row split; wave w owns columns [16w, 16w+16): TAPS x 4 accumulators.
// partial[split][t][k][n]; reduced over splits in a fixed order by reduce_kernel.
constexpr int GK = 64, GN = 64, GR = 64, GS = 80;

// NB independent problems (X + i xbs, DY + i dbs: the 16 Winograd points of a weight grad) share
// one launch: blockIdx.z = problem * splits + split, partial[split][problem][t][k][n].
// KI: the 16-channel k blocks of the tile that hold data (4; 2 for the input conv's 32 padded
// channels, whose upper half would only multiply zeros)
template <int TAPS, int KI = 4>
__global__ void __launch_bounds__(256)
wgrad_f32_kernel(const float* __restrict__ X, int ldx, int K, const float* __restrict__ DY, int ldd, int N, int R,
                 int rows_per_split, float* __restrict__ partial, int nb, size_t xbs, size_t dbs) {
    __shared__ __attribute__((aligned(16))) float xs[GR * GS + GS];
    __shared__ __attribute__((aligned(16))) float ds[GR * GS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int splits = gridDim.z / nb, split = blockIdx.z % splits, pb = blockIdx.z / splits;
    const int k0 = blockIdx.x * GK, n0 = blockIdx.y * GN;
    X += pb * xbs;
    DY += pb * dbs;
    const int rbeg = split * rows_per_split, rend = min(R, rbeg + rows_per_split);
    f32x4 acc[TAPS][KI];
#pragma unroll
    for (int t = 0; t < TAPS; t++)
#pragma unroll
        for (int i = 0; i < KI; i++) acc[t][i] = f32x4{0, 0, 0, 0};
    if (tid < GS) xs[GR * GS + tid] = 0.0f;
    // software pipeline: the next GR rows of X and dY are read into registers while the current
    // rows' MFMAs run, and written to LDS after the barrier
    constexpr int NV = GR * 16 / 256;
    float4 xv[NV], dv[NV];
    auto fetch = [&](int rc) {
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int i = tid + j * 256, rr = i >> 4, c4 = (i & 15) * 4;
            xv[j] = dv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (rc + rr < rend) {
                if (c4 < 16 * KI && k0 + c4 < K) xv[j] = *reinterpret_cast<const float4*>(X + (size_t)(rc + rr) * ldx + k0 + c4);
                if (n0 + c4 < N) dv[j] = *reinterpret_cast<const float4*>(DY + (size_t)(rc + rr) * ldd + n0 + c4);
            }
        }
    };
    if (rbeg < rend) fetch(rbeg);
    for (int rc = rbeg; rc < rend; rc += GR) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int i = tid + j * 256, rr = i >> 4, c4 = (i & 15) * 4;
            *reinterpret_cast<float4*>(xs + rr * GS + c4) = xv[j];
            *reinterpret_cast<float4*>(ds + rr * GS + c4) = dv[j];
        }
        __syncthreads();
        if (rc + GR < rend) fetch(rc + GR);
#pragma unroll 2
        for (int q = 0; q < GR / 4; q++) {
            const int rq = q * 4 + (lane >> 4);
            const float b = ds[rq * GS + w * 16 + (lane & 15)];
#pragma unroll
            for (int t = 0; t < TAPS; t++) {
                int src = rq;
                bool ok = true;
                if constexpr (TAPS == 9) ok = tap_src(rq, t, src);
                const int base = ok ? src * GS : GR * GS;
#pragma unroll
                for (int i = 0; i < KI; i++)
                    acc[t][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[base + i * 16 + (lane & 15)], b, acc[t][i], 0, 0, 0);
            }
        }
    }
    const int n = n0 + w * 16 + (lane & 15);
    if (n >= N) return;
#pragma unroll
    for (int t = 0; t < TAPS; t++)
#pragma unroll
        for (int i = 0; i < KI; i++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int kd = k0 + i * 16 + (lane >> 4) * 4 + g;
                if (kd < K) partial[((((size_t)split * nb + pb) * TAPS + t) * K + kd) * N + n] = acc[t][i][g];
            }
}

// Winograd weight grad at F = 256, transforms fused into the GEMM's staging: one workgroup per
// (split of 512 (board, tile) rows, point xi = 4 r + q) computes the whole 256 x 256 dU[xi] partial
// over its rows.  Each stage is one board: the workgroup gathers the 2 x 2 input squares and the
// 2 x 2 output-gradient squares point xi combines per (tile, channel) -- V[xi] = (B^T d B)[r][q]
// and M'[xi] = (A dY A^T)[r][q] with the same additions in the same order as the
// round-3 transform pass (now tools/wgrad_dbg.hip) -- straight from X and dY (the 16 point workgroups of a split share
// one XCD's L2: workgroup id = split + splits xi), so the 16 transformed operands never go to HBM.
// GEMM: 8 waves, wave w owns co [32 w, 32 w + 32) x all 256 ci: accumulator block (j, c) row m is
// ci = 64 j + 4 m + c, so one ds_read_b128 of a row feeds four blocks.  The next board's squares
// are loaded into registers beside the current board's MFMAs.  partial[split][xi][ci][co]; every
// element sums its split's rows in row order (fixed order; splits reduced in order by
// wino_wgrad_reduce_out_kernel).
// LDS row strides (floats): V rows are read by ds_read_b128 (lane groups {0-3,12-15,20-27}, ...:
// two rows per group, conflict-free when the rows are 0 mod 64 banks apart), M' rows by
// ds_read_b32 (32-lane groups over two rows, conflict-free when 16 mod 32 apart).  One stride of
// 272 for both measured 36 % of LDS cycles as bank conflicts (profiles/r04g_pmc_train_wino_wgrad_gemm.json).
constexpr int WG_SX = 256, WG_SD = 256 + 16;
// the four F(2x2,3x3) combinations: (a, b) = (e0, e2) / (e1, e2) / (e1, e2) / (e1, e3) of a patch
// row or column -> a - b, a + b, b - a, a - b (B^T rows)
__device__ __forceinline__ f32x4 wino_comb(int k, f32x4 a, f32x4 b) { return k == 1 ? a + b : k == 2 ? b - a : a - b; }
// (16 waves of 16 output channels each, 4 per SIMD at <= 128 VGPRs, measured the same: 166.1 vs
// 166.7 us, profiles/r04g_train_kernel_stats_w16.csv; not kept.  Round 5: double-buffered staging
// with one barrier per board, the next board's transform between the row quads' MFMAs -- 22.68 /
// 22.57 ms per step (transform mid-board / after the last quad) against 22.35 -- and a
// branch-free sign-mask form of wino_comb, 23.21: both spill (4-12 VGPRs) at the 256-VGPR cap;
// profiles/r05h_train_ab.txt.  Not kept.)
// (Round 6: X by LDS-DMA into a raw board image of only the point's distinct squares -- a corner
// point's workgroup then issues 16 X loads per board instead of 64, 576 instead of 1,024 per split
// and board -- bit-identical, measured 22.43 vs 21.93 ms per step at B = 512 and flat at 64,
// profiles/r06h_ab_glds_b512.txt: the per-board vmcnt(0) drain at the staging barrier and the
// image's LDS reads cost more than the load instructions saved.  Not kept.)
__global__ void __launch_bounds__(512)
wino_wgrad_gemm_kernel(const float* __restrict__ X, const float* __restrict__ DY, int K, int rows_per_split,
                       float* __restrict__ partial) {
    constexpr int NWG = 8, F = 256, CO = F / NWG, NN = CO / 16, TPT = 16 / NWG;
    __shared__ __attribute__((aligned(16))) float xs[16 * WG_SX];
    __shared__ __attribute__((aligned(16))) float ds[16 * WG_SD];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int split = blockIdx.x, xi = blockIdx.y, r = xi >> 2, q = xi & 3;
    const int i1 = r == 0 ? 0 : 1, i2 = r == 3 ? 3 : 2, j1 = q == 0 ? 0 : 1, j2 = q == 3 ? 3 : 2;
    const int rbeg = split * rows_per_split, rend = min(K, rbeg + rows_per_split);
    f32x4 acc[16][NN];
#pragma unroll
    for (int b = 0; b < 16; b++)
#pragma unroll
        for (int n = 0; n < NN; n++) acc[b][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // staging: thread = (channel quad c4, tiles TPT tp .. TPT tp + TPT - 1).  The squares come in
    // through buffer loads: the lane's channel offset is the only VGPR address, the (wave-uniform)
    // square offset rides in the SGPR offset, and an off-board square moves the VGPR offset past
    // the buffer's end (the range check covers the VGPR offset), which the hardware reads as 0 (no
    // branch, no 64-bit address per load)
    const int c4 = (tid & 63) * 4, tp = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int xbytes = (K >> 4) * 64 * F * 4;   // K (board, tile) rows = K / 16 boards
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc((void*)DY, (short)0, xbytes, 0x00020000);
    constexpr int OFF_BOARD = 0x40000000;       // past any buffer this kernel is given (< 1 GiB, host-checked)
    f32x4 xd[TPT][2][2], yv[TPT][2][2];   // [tile][patch row i1 / i2][patch column j1 / j2], [tile][a][b]
    auto fetch = [&](int rc) {
        const int bb0 = (rc >> 4) * 64 * F * 4;
#pragma unroll
        for (int u = 0; u < TPT; u++) {
            const int t = TPT * tp + u, ty = t >> 2, tx = t & 3;
#pragma unroll
            for (int ii = 0; ii < 2; ii++)
#pragma unroll
                for (int jj = 0; jj < 2; jj++) {
                    const int row = 2 * ty - 1 + (ii ? i2 : i1), col = 2 * tx - 1 + (jj ? j2 : j1);
                    const bool on = (unsigned)row < 8u && (unsigned)col < 8u;
                    xd[u][ii][jj] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                  rX, on ? c4 * 4 : OFF_BOARD, on ? bb0 + (row * 8 + col) * F * 4 : 0, 0));
                }
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int bb = 0; bb < 2; bb++)
                    yv[u][a][bb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                 rD, c4 * 4, bb0 + ((2 * ty + a) * 8 + 2 * tx + bb) * F * 4, 0));
        }
    };
    if (rbeg < rend) fetch(rbeg);
    for (int rc = rbeg; rc < rend; rc += 16) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < TPT; u++) {
            const int t = TPT * tp + u;
            // V: rows first (tt over the two columns), then the column combination
            const f32x4 tt1 = wino_comb(r, xd[u][0][0], xd[u][1][0]), tt2 = wino_comb(r, xd[u][0][1], xd[u][1][1]);
            const f32x4 v = wino_comb(q, tt1, tt2);
            // M': p_b = (A dY)[r][b], then (p A^T)[q], as ca y0 + cb y1 with the rows of A
            // {(1, 0), (1, 1), (1, -1), (0, -1)}: every product is by 1, -1 or 0, so the values are
            // the transform kernel's (signed zeros aside).  The same as a select chain
            // (r == 0 ? y0 : ... : -y1) was miscompiled for gfx950: r = 3 produced y0 on the GPU
            // (tools/wgrad_dbg.hip, profiles/r04_wgrad_dbg.log), while a CPU emulation was right.
            const float ra = r == 3 ? 0.0f : 1.0f, rb = r == 0 ? 0.0f : (r == 1 ? 1.0f : -1.0f);
            const float qa = q == 3 ? 0.0f : 1.0f, qb = q == 0 ? 0.0f : (q == 1 ? 1.0f : -1.0f);
            f32x4 p[2];
#pragma unroll
            for (int bb = 0; bb < 2; bb++) p[bb] = yv[u][0][bb] * ra + yv[u][1][bb] * rb;
            const f32x4 m = p[0] * qa + p[1] * qb;
            *reinterpret_cast<f32x4*>(xs + t * WG_SX + c4) = v;
            *reinterpret_cast<f32x4*>(ds + t * WG_SD + c4) = m;
        }
        __syncthreads();
        if (rc + 16 < rend) fetch(rc + 16);
        // the operands of row quad qq + 1 are read while the MFMAs of qq run (read just in time,
        // every 8 MFMAs waited on an LDS round trip: 62 % matrix-pipe busy, PMC)
        float bA[NN], bB[NN];
        f32x4 aA[4], aB[4];
        auto rd = [&](int qq, float (&bv)[NN], f32x4 (&av)[4]) {
            const int rq = qq * 4 + (lane >> 4);
#pragma unroll
            for (int n = 0; n < NN; n++) bv[n] = ds[rq * WG_SD + CO * w + 16 * n + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 4; j++) av[j] = *reinterpret_cast<const f32x4*>(xs + rq * WG_SX + 64 * j + 4 * (lane & 15));
        };
        auto mm = [&](const float (&bv)[NN], const f32x4 (&av)[4]) {
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int c = 0; c < 4; c++)
#pragma unroll
                    for (int n = 0; n < NN; n++)
                        acc[4 * j + c][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j][c], bv[n], acc[4 * j + c][n], 0, 0, 0);
        };
        rd(0, bA, aA);
        rd(1, bB, aB);
        __builtin_amdgcn_sched_barrier(0);
        mm(bA, aA);
        __builtin_amdgcn_sched_barrier(0);
        rd(2, bA, aA);
        __builtin_amdgcn_sched_barrier(0);
        mm(bB, aB);
        __builtin_amdgcn_sched_barrier(0);
        rd(3, bB, aB);
        __builtin_amdgcn_sched_barrier(0);
        mm(bA, aA);
        __builtin_amdgcn_sched_barrier(0);
        mm(bB, aB);
    }
    float* out = partial + ((size_t)split * 16 + xi) * F * F;
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int n = 0; n < NN; n++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int ci = 64 * j + 4 * (4 * (lane >> 4) + g) + c, co = CO * w + 16 * n + (lane & 15);
                    out[(size_t)ci * F + co] = acc[4 * j + c][n][g];
                }
}

// f(std::integral_constant<int, I>) for I = 0 .. N-1, unrolled by construction (a #pragma unroll over
// the weight grad's 256-MFMA board with its side jobs was left rolled, and its indexed register
// arrays went to scratch)
template <class Fn, int... Is>
__device__ __forceinline__ void static_for_impl(Fn&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& f) { static_for_impl(f, std::make_integer_sequence<int, N>{}); }
// The same weight grad with one wave per SIMD (round 6, the default): 4 waves, wave w owns co
// [64 w, 64 w + 64) x all 256 ci -- 256 accumulators per lane, in AGPRs, updated in place by inline
// asm MFMAs (with the builtin, 256 live accumulators made the allocator copy them between AGPRs
// and VGPRs every board) -- and the transformed board in two LDS buffers.  While board b's MFMAs
// run from one buffer, the wave transforms board b + 1's squares (loaded a board earlier) into the
// other and issues board b + 2's loads into the registers just freed, in small steps between single
// MFMAs, so that per board only one barrier and the first quad's LDS reads are exposed.  The point
// (r, q) is a template parameter (one body per point, chosen by blockIdx.y), so a transform step is
// four adds.  Every accumulator gets the same MFMA sequence as in wino_wgrad_gemm_kernel (rows in
// order, four per MFMA) and the transforms the same operations: the partials are bit-identical
// (test_weight_grad_one_wave_per_simd_bit_identical).  Measured at B = 512
// (profiles/r06u_ab_wgrad4_b512.txt, r06o_wgrad_pricing.txt): 148.6 us against 164-168 us, and
// 130.9 us with the side jobs removed (a pricing build, wrong results): the transforms and loads
// cost the one MFMA wave ~12 %, which fillers of 16-24 cycles per 32-cycle f32 MFMA gap do not hide.
template <int R, int Q, int NQ>
__device__ __forceinline__ void wgrad4_body(const float* __restrict__ X, const float* __restrict__ DY, int K,
                                            int rows_per_split, float* __restrict__ partial, float* xsm, float* dsm) {
    // NQ output-channel parts per (split, point): the workgroup owns co [FQ z, FQ z + FQ) (blockIdx.z)
    constexpr int NWV = 4, F = 256, FQ = F / NQ, CO = FQ / NWV, NN = CO / 16, TPT = 16 / NWV;
    constexpr int MQ = FQ / 4, MIT = 16 * MQ / 256;   // M' items (tile, co quad) per thread: 4 / NQ
    constexpr int XB = 16 * WG_SX, DB = 16 * WG_SD;   // one LDS buffer of V / M' rows
    constexpr int I1 = R == 0 ? 0 : 1, I2 = R == 3 ? 3 : 2, J1 = Q == 0 ? 0 : 1, J2 = Q == 3 ? 3 : 2;
    constexpr float RA = R == 3 ? 0.0f : 1.0f, RB = R == 0 ? 0.0f : (R == 1 ? 1.0f : -1.0f);
    constexpr float QA = Q == 3 ? 0.0f : 1.0f, QB = Q == 0 ? 0.0f : (Q == 1 ? 1.0f : -1.0f);
    static_assert(NN >= 1 && MIT >= 1 && 4 % MIT == 0, "co parts");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int split = blockIdx.x, cob = FQ * (int)blockIdx.z;
    const int rbeg = split * rows_per_split, rend = min(K, rbeg + rows_per_split), nbd = (rend - rbeg) >> 4;
    f32x4 acc[16][NN];
#pragma unroll
    for (int b = 0; b < 16; b++)
#pragma unroll
        for (int n = 0; n < NN; n++) acc[b][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int c4 = lane * 4, tp = __builtin_amdgcn_readfirstlane(w);
    const int xbytes = (K >> 4) * 64 * F * 4;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc((void*)DY, (short)0, xbytes, 0x00020000);
    constexpr int OFF_BOARD = 0x40000000;
    f32x4 xd[TPT][2][2], yv[MIT][2][2];
    // wino_comb and the M' combination of wino_wgrad_gemm_kernel with the point's constants, in
    // steps of four floats (so that one step fits beside one MFMA): V of tile u (the thread's
    // channel quad lane of all 256 input channels), M' of item m (tile (tid + 256 m) / MQ, output
    // channel quad (tid + 256 m) % MQ of the workgroup's FQ)
    f32x4 t1[TPT], t2[TPT], p0[MIT], p1[MIT];
    auto vstep = [&](int buf, int u, int st) {
        const int t = TPT * tp + u;
        if (st == 0) t1[u] = wino_comb(R, xd[u][0][0], xd[u][1][0]);
        if (st == 1) t2[u] = wino_comb(R, xd[u][0][1], xd[u][1][1]);
        if (st == 2) *reinterpret_cast<f32x4*>(xsm + buf * XB + t * WG_SX + c4) = wino_comb(Q, t1[u], t2[u]);
    };
    auto mstep = [&](int buf, int m, int st) {
        const int idx = tid + 256 * m, t = idx / MQ, cq = idx % MQ;
        if (st == 0) p0[m] = yv[m][0][0] * RA + yv[m][1][0] * RB;
        if (st == 1) p1[m] = yv[m][0][1] * RA + yv[m][1][1] * RB;
        if (st == 2) *reinterpret_cast<f32x4*>(dsm + buf * DB + t * WG_SD + 4 * cq) = p0[m] * QA + p1[m] * QB;
    };
    // X square i (0-3) of tile u, dY square i (0-3) of item m, of board bi (bi >= nbd: zeros, no branch)
    auto loadx = [&](int bi, int u, int i) {
        const bool inb = bi < nbd;
        const int bb0 = inb ? ((rbeg >> 4) + bi) * 64 * F * 4 : 0, vin = inb ? c4 * 4 : OFF_BOARD;
        const int t = TPT * tp + u, ty = t >> 2, tx = t & 3;
        const int ii = i >> 1, jj = i & 1;
        const int row = 2 * ty - 1 + (ii ? I2 : I1), col = 2 * tx - 1 + (jj ? J2 : J1);
        const bool on = (unsigned)row < 8u && (unsigned)col < 8u;
        xd[u][ii][jj] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rX, on ? vin : OFF_BOARD, on ? bb0 + (row * 8 + col) * F * 4 : 0, 0));
    };
    auto loady = [&](int bi, int m, int i) {
        const bool inb = bi < nbd;
        const int idx = tid + 256 * m, t = idx / MQ, cq = idx % MQ, ty = t >> 2, tx = t & 3;
        const int a = i >> 1, bb = i & 1;
        const int bb0 = inb ? ((rbeg >> 4) + bi) * 64 * F * 4 : 0;
        const int vo = inb ? (((2 * ty + a) * 8 + 2 * tx + bb) * F + cob + 4 * cq) * 4 : OFF_BOARD;
        yv[m][a][bb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rD, vo, bb0, 0));
    };
    if (nbd > 0) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
#pragma unroll
            for (int u = 0; u < TPT; u++) loadx(0, u, i);
#pragma unroll
            for (int m = 0; m < MIT; m++) loady(0, m, i);
        }
#pragma unroll
        for (int st = 0; st < 3; st++) {
#pragma unroll
            for (int u = 0; u < TPT; u++) vstep(0, u, st);
#pragma unroll
            for (int m = 0; m < MIT; m++) mstep(0, m, st);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
#pragma unroll
            for (int u = 0; u < TPT; u++) loadx(1, u, i);
#pragma unroll
            for (int m = 0; m < MIT; m++) loady(1, m, i);
        }
    }
    __syncthreads();
    float bv[2][NN];
    f32x4 av[2][4];
    // side-job slots in a row quad of 16 NN MFMAs: the V steps VS MFMAs apart from k = 0, the M'
    // steps from k = 3 VS, then the eight loads LS MFMAs apart from k = L0 (a load costs the issuing
    // wave more than one MFMA gap, so they are spread over the quad)
    constexpr int VS = NN >= 2 ? 2 : 1, L0 = NN >= 4 ? 16 : NN == 2 ? 12 : 6, LS = NN >= 4 ? 6 : NN == 2 ? 2 : 1;
    static_assert(L0 + 7 * LS < 16 * NN && 6 * VS <= L0, "side-job slots fit the quad");
    for (int b = 0; b < nbd; b++) {
        const int cur = b & 1, nxt = cur ^ 1;
        auto rd = [&](int qq) {
            const int rq = qq * 4 + (lane >> 4), o = qq & 1;
#pragma unroll
            for (int n = 0; n < NN; n++) bv[o][n] = dsm[cur * DB + rq * WG_SD + CO * w + 16 * n + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 4; j++) av[o][j] = *reinterpret_cast<const f32x4*>(xsm + cur * XB + rq * WG_SX + 64 * j + 4 * (lane & 15));
        };
        // beside row quad u: board b + 1's V of tile u and M' of item u / (4 / MIT) (in the quads
        // u % (4 / MIT) == 0), then board b + 2's loads of them into the registers just freed
        auto side = [&](auto U, auto KK) {
            constexpr int u = decltype(U)::value, k = decltype(KK)::value;
            constexpr bool hasm = u % (4 / MIT) == 0;
            constexpr int m = u / (4 / MIT);
            if constexpr (k < 3 * VS && k % VS == 0) vstep(nxt, u, k / VS);
            if constexpr (hasm && k >= 3 * VS && k < 6 * VS && k % VS == 0) mstep(nxt, m, (k - 3 * VS) / VS);
            if constexpr (k >= L0 && (k - L0) % LS == 0 && (k - L0) / LS < 4) loadx(b + 2, u, (k - L0) / LS);
            if constexpr (hasm && k >= L0 && (k - L0) % LS == 0 && (k - L0) / LS >= 4 && (k - L0) / LS < 8)
                loady(b + 2, m, (k - L0) / LS - 4);
        };
        rd(0);
        static_for<16>([&](auto G) {
            constexpr int g = decltype(G)::value, qq = g >> 2, j = g & 3, o = qq & 1;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g == 0) rd(1);
            if constexpr (g == 4) rd(2);
            if constexpr (g == 8) rd(3);
            __builtin_amdgcn_sched_barrier(0);
            static_for<4 * NN>([&](auto CN) {
                constexpr int c = decltype(CN)::value / NN, n = decltype(CN)::value % NN, k = 4 * NN * j + NN * c + n;
                asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc[4 * j + c][n]) : "v"(av[o][j][c]), "v"(bv[o][n]));
                if constexpr ((k < 6 * VS && k % VS == 0) || (k >= L0 && (k - L0) % LS == 0 && (k - L0) / LS < 8)) {
                    __builtin_amdgcn_sched_barrier(0);
                    side(std::integral_constant<int, qq>{}, std::integral_constant<int, k>{});
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
        });
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
    }
    // the MFMAs are inline asm: the compiler does not count their latency before the AGPR reads
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    float* out = partial + ((size_t)split * 16 + 4 * R + Q) * F * F;
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int n = 0; n < NN; n++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int ci = 64 * j + 4 * (4 * (lane >> 4) + g) + c, co = cob + CO * w + 16 * n + (lane & 15);
                    out[(size_t)ci * F + co] = acc[4 * j + c][n][g];
                }
}
template <int NQ>
__global__ void __launch_bounds__(256)
wino_wgrad_gemm4_kernel(const float* __restrict__ X, const float* __restrict__ DY, int K, int rows_per_split,
                        float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float xs[2 * 16 * WG_SX];
    __shared__ __attribute__((aligned(16))) float ds[2 * 16 * WG_SD];
#define AZ_WG4(x) case x: wgrad4_body<((x) / 4), ((x) % 4), NQ>(X, DY, K, rows_per_split, partial, xs, ds); break;
    switch (blockIdx.y) {
        AZ_WG4(0) AZ_WG4(1) AZ_WG4(2) AZ_WG4(3) AZ_WG4(4) AZ_WG4(5) AZ_WG4(6) AZ_WG4(7)
        AZ_WG4(8) AZ_WG4(9) AZ_WG4(10) AZ_WG4(11) AZ_WG4(12) AZ_WG4(13) AZ_WG4(14) AZ_WG4(15)
    }
#undef AZ_WG4
}

// out[e] = sum over splits s (in order) of partial[s][e]
__global__ void reduce_kernel(const float* __restrict__ partial, int splits, size_t n, float* __restrict__ out) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        float s = 0.0f;   // (the splits' loads 8 at a time, added in order: see wino_wgrad_reduce_out_kernel)
        for (int k0 = 0; k0 < splits; k0 += 8) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = partial[(size_t)min(k0 + j, splits - 1) * n + e];
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (k0 + j < splits) s += v[j];
        }
        out[e] = s;
    }
}

// ------------------------------------------------------------------ column reductions
// Per-channel sums over rows, fixed order: block (x = row block, y = 64-channel block); thread
// (phase p = tid/64, channel c) sums rows rbeg+p, rbeg+p+4, ...; phases are combined in order.
//   MODE 0: sum v                       (bias grads, BN mean)
//   MODE 1: sum (v - mean)^2            (BN biased variance, two-pass like burn)
//   MODE 2: sum dz, sum dz*yhat with dz = dout*(o > 0), yhat = (y - mean)/std   (BN backward)
constexpr int CS_ROWS = 256;   // rows per block

template <int MODE>
__global__ void __launch_bounds__(256)
colsum_kernel(const float* __restrict__ V, int ld, int C, int R, const float* __restrict__ mean,
              const float* __restrict__ stdv, const float* __restrict__ O, const float* __restrict__ Y,
              float* __restrict__ part) {
    __shared__ float sh[2][4][64];
    const int tid = threadIdx.x, p = tid >> 6, c = blockIdx.y * 64 + (tid & 63);
    const int rbeg = blockIdx.x * CS_ROWS, rend = min(R, rbeg + CS_ROWS);
    float s0 = 0.0f, s1 = 0.0f;
    if (c < C) {
        const float mu = (MODE >= 1) ? mean[c] : 0.0f;
        const float sd = (MODE == 2) ? stdv[c] : 1.0f;
#pragma unroll 4
        for (int r = rbeg + p; r < rend; r += 4) {
            const size_t e = (size_t)r * ld + c;
            if constexpr (MODE == 0) {
                s0 += V[e];
            } else if constexpr (MODE == 1) {
                const float d = V[e] - mu;
                s0 += d * d;
            } else {
                const float dz = O[e] > 0.0f ? V[e] : 0.0f;
                s0 += dz;
                s1 += dz * ((Y[e] - mu) / sd);
            }
        }
    }
    sh[0][p][tid & 63] = s0;
    sh[1][p][tid & 63] = s1;
    __syncthreads();
    if (p == 0 && c < C) {
        const float a = ((sh[0][0][tid] + sh[0][1][tid]) + sh[0][2][tid]) + sh[0][3][tid];
        part[((size_t)blockIdx.x * 2 + 0) * C + c] = a;
        if (MODE == 2) part[((size_t)blockIdx.x * 2 + 1) * C + c] = ((sh[1][0][tid] + sh[1][1][tid]) + sh[1][2][tid]) + sh[1][3][tid];
    }
}

// What becomes of a column sum (the finalize kernels below):  SUM a = s0;  MEAN a = s0 / R;  VAR
// var = s0 / R, a = sqrt(var + eps), b = running mean, c = running var (momentum 0.1, batch mean
// `mean`);  BNBACK a = dgamma = s1, b = dbeta = s0.
enum { FIN_SUM, FIN_MEAN, FIN_VAR, FIN_BNBACK };
struct ColFin {
    int kind;
    float *a, *b, *c;
    const float* mean;
};

// The same sums four channels per thread (16-byte loads; C and ld multiples of 4): thread
// (phase p = tid / 16, quad q = tid % 16) sums rows rbeg + p, rbeg + p + 16, ... of channels
// 64 blockIdx.y + 4 q .. + 3, phases combined in order.  16 phases instead of 4 keep 4x more loads in
// flight (MODE 2, three streams and a division per element: 41 -> ? us per launch at 32768 x 256).
template <int MODE>
__global__ void __launch_bounds__(256)
colsum4_kernel(const float* __restrict__ V, int ld, int C, int R, const float* __restrict__ mean,
               const float* __restrict__ stdv, const float* __restrict__ O, const float* __restrict__ Y,
               float* __restrict__ part) {
    __shared__ float4 sh[2][16][16];
    const int tid = threadIdx.x, p = tid >> 4, q = tid & 15, c = blockIdx.y * 64 + 4 * q;
    const int rbeg = blockIdx.x * CS_ROWS, rend = min(R, rbeg + CS_ROWS);
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    if (c < C) {
        const float4 mu = (MODE >= 1) ? *reinterpret_cast<const float4*>(mean + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 sd = (MODE == 2) ? *reinterpret_cast<const float4*>(stdv + c) : make_float4(1.f, 1.f, 1.f, 1.f);
#pragma unroll 4
        for (int r = rbeg + p; r < rend; r += 16) {
            const size_t e = (size_t)r * ld + c;
            const float4 v = *reinterpret_cast<const float4*>(V + e);
            if constexpr (MODE == 0) {
                s0.x += v.x; s0.y += v.y; s0.z += v.z; s0.w += v.w;
            } else if constexpr (MODE == 1) {
                const float dx = v.x - mu.x, dy = v.y - mu.y, dz = v.z - mu.z, dw = v.w - mu.w;
                s0.x += dx * dx; s0.y += dy * dy; s0.z += dz * dz; s0.w += dw * dw;
            } else {
                const float4 o = *reinterpret_cast<const float4*>(O + e), y = *reinterpret_cast<const float4*>(Y + e);
                const float zx = o.x > 0.0f ? v.x : 0.0f, zy = o.y > 0.0f ? v.y : 0.0f;
                const float zz = o.z > 0.0f ? v.z : 0.0f, zw = o.w > 0.0f ? v.w : 0.0f;
                s0.x += zx; s0.y += zy; s0.z += zz; s0.w += zw;
                s1.x += zx * ((y.x - mu.x) / sd.x); s1.y += zy * ((y.y - mu.y) / sd.y);
                s1.z += zz * ((y.z - mu.z) / sd.z); s1.w += zw * ((y.w - mu.w) / sd.w);
            }
        }
    }
    sh[0][p][q] = s0;
    sh[1][p][q] = s1;
    __syncthreads();
    if (tid < 64) {                                    // thread = channel blockIdx.y * 64 + tid
        const int cq = tid >> 2, k = tid & 3, cc = blockIdx.y * 64 + tid;
        if (cc < C) {
            const int nw = MODE == 2 ? 2 : 1;
            for (int wch = 0; wch < nw; wch++) {
                float a = 0.0f;
                for (int ph = 0; ph < 16; ph++) a += reinterpret_cast<const float*>(&sh[wch][ph][cq])[k];
                part[((size_t)blockIdx.x * 2 + wch) * C + cc] = a;
            }
        }
    }
}


// sum the row-block partials of channel c, one wavefront per channel: lane l adds blocks
// l, l + 64, ... in order, then a fixed butterfly over the lanes -- a fixed order (the step stays
// bit-reproducible), 64 loads in flight instead of one dependent chain of nblk.  Each lane's loads
// go out 8 at a time and are added in block order after they land (round 6: the loop issued one
// load per round trip -- 8 dependent L2 trips for 512 boards, most of these kernels' 8 us)
constexpr int PSUM_BATCH = 8;
// one chunk of a lane's blocks, b0 + 64 k for k < NK: all loads first (past the end: the last block,
// loaded and not added), then the adds in block order
template <int NW, int NK>
__device__ __forceinline__ void part_chunk(const float* part, int nblk, int C, int c, const int (&which)[NW], int b0,
                                           float (&s)[NW]) {
    float v[NW][NK];
#pragma unroll
    for (int k = 0; k < NK; k++)
#pragma unroll
        for (int q = 0; q < NW; q++) v[q][k] = part[((size_t)min(b0 + 64 * k, nblk - 1) * 2 + which[q]) * C + c];
#pragma unroll
    for (int k = 0; k < NK; k++)
#pragma unroll
        for (int q = 0; q < NW; q++) s[q] = b0 + 64 * k < nblk ? s[q] + v[q][k] : s[q];
}
// the butterfly s += shfl_xor(s, m), m = 32 .. 1, of a wavefront's 64 lanes, over the 64 lanes of
// a channel in a finalize workgroup (FIN_CHANNEL) through LDS: level m adds lane l + m into lane l,
// l < m -- lane 0's operands at every level, so the same bits (the butterfly leaves every lane with
// lane 0's value: x + y = y + x exactly).  Every thread of the workgroup calls it.
__device__ __forceinline__ float lane_butterfly(float s) {
    __shared__ float red[64][17];
    const int lane = threadIdx.x >> 4, j = threadIdx.x & 15;
    __syncthreads();   // the previous call's readers are done
    red[lane][j] = s;
    __syncthreads();
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        if (lane < m) red[lane][j] = red[lane][j] + red[lane + m][j];
        __syncthreads();
    }
    return red[0][j];
}
template <int NW>
__device__ __forceinline__ void part_sums(const float* part, int nblk, int C, int c, const int (&which)[NW], int lane,
                                          float (&s)[NW]) {
#pragma unroll
    for (int q = 0; q < NW; q++) s[q] = 0.0f;
    if (nblk <= 64) part_chunk<NW, 1>(part, nblk, C, c, which, lane, s);
    else
        for (int b0 = lane; b0 < nblk; b0 += 64 * PSUM_BATCH) part_chunk<NW, PSUM_BATCH>(part, nblk, C, c, which, b0, s);
#pragma unroll
    for (int q = 0; q < NW; q++) s[q] = lane_butterfly(s[q]);
}
__device__ __forceinline__ float part_sum(const float* part, int nblk, int C, int c, int which, int lane) {
    float s[1];
    part_sums<1>(part, nblk, C, c, {which}, lane, s);
    return s[0];
}
// BN forward statistics of channel c from per-board partials (BoardStats STATS 1): the sum S and
// sum_b [M2_b + 64 (S_b / 64 - S / R)^2] (Chan et al.'s pairwise update, every board 64 rows), both
// in part_sum's order.  Up to 512 boards from one set of loads (the mean's butterfly, then the
// deviations from the same registers); more in two passes.
template <int NK>
__device__ __forceinline__ void board_stats_regs(const float* part, int nb, int C, int c, int R, int lane, float& s,
                                                 float& m2) {
    float vs[NK], vm[NK];
#pragma unroll
    for (int k = 0; k < NK; k++) {
        const int b = min(lane + 64 * k, nb - 1);
        vs[k] = part[((size_t)b * 2) * C + c];
        vm[k] = part[((size_t)b * 2 + 1) * C + c];
    }
    s = 0.0f;
#pragma unroll
    for (int k = 0; k < NK; k++) s = lane + 64 * k < nb ? s + vs[k] : s;
    s = lane_butterfly(s);
    const float mu = s / (float)R;
    m2 = 0.0f;
#pragma unroll
    for (int k = 0; k < NK; k++) {
        const float d = vs[k] / 64.0f - mu;
        const float t = m2 + (vm[k] + 64.0f * (d * d));
        m2 = lane + 64 * k < nb ? t : m2;
    }
    m2 = lane_butterfly(m2);
}
__device__ __forceinline__ void board_stats(const float* part, int nb, int C, int c, int R, int lane, float& s, float& m2) {
    if (nb <= 64) return board_stats_regs<1>(part, nb, C, c, R, lane, s, m2);
    if (nb <= 64 * PSUM_BATCH) return board_stats_regs<PSUM_BATCH>(part, nb, C, c, R, lane, s, m2);
    s = part_sum(part, nb, C, c, 0, lane);
    const float mu = s / (float)R;
    m2 = 0.0f;
    for (int b = lane; b < nb; b += 64) {
        const float d = part[((size_t)b * 2) * C + c] / 64.0f - mu;
        m2 += part[((size_t)b * 2 + 1) * C + c] + 64.0f * (d * d);
    }
    m2 = lane_butterfly(m2);
}
// workgroup = 16 channels x 64 lanes (launch finalize_grid(C) blocks of FIN_THREADS): thread
// (lane tid >> 4, channel 16 blockIdx.x + tid % 16), so that 16 neighbouring threads read one 64-byte
// run of a partials row.  (Round 6: one wavefront per channel read 4 useful bytes per 64-byte line,
// 16 lines per run; the step's batched bias sums took 32.6 us.)  Channels past C load channel C - 1
// and write nothing; every thread reaches the butterflies' barriers.
constexpr int FIN_THREADS = 1024;
inline int finalize_grid(int C) { return (C + 15) / 16; }
#define FIN_CHANNEL()                                                            \
    const int lane = threadIdx.x >> 4;                                           \
    const bool cown = (int)(16 * blockIdx.x + (threadIdx.x & 15)) < C;           \
    const int c = min((int)(16 * blockIdx.x + (threadIdx.x & 15)), C - 1)

// dst[c] = sum  (bias gradients)
__global__ void finalize_sum_kernel(const float* __restrict__ part, int nblk, int C, float* __restrict__ dst) {
    FIN_CHANNEL();
    const float s = part_sum(part, nblk, C, c, 0, lane);
    if (lane == 0 && cown) dst[c] = s;
}

// the bias gradients of every BN-fed conv of the step in one launch (they are needed only by the
// optimizer): blockIdx.y = BatchNorm j, its bn_back4 partials at part + j pstride, its gradient at
// g + dst[j]
__global__ void finalize_sum_batched_kernel(const float* __restrict__ part, size_t pstride, int nblk, int C,
                                            const uint32_t* __restrict__ dst, float* __restrict__ g) {
    FIN_CHANNEL();
    const float s = part_sum(part + blockIdx.y * pstride, nblk, C, c, 0, lane);
    if (lane == 0 && cown) g[dst[blockIdx.y] + c] = s;
}

// mean[c] = sum / R
__global__ void finalize_mean_kernel(const float* __restrict__ part, int nblk, int C, int R, float* __restrict__ mean) {
    FIN_CHANNEL();
    const float s = part_sum(part, nblk, C, c, 0, lane);
    if (lane == 0 && cown) mean[c] = s / (float)R;
}

// var = sum / R; std = sqrt(var + eps); running stats: rm = rm*0.9 + mean*0.1, rv = rv*0.9 + var*0.1
__global__ void finalize_var_kernel(const float* __restrict__ part, int nblk, int C, int R, const float* __restrict__ mean,
                                    float* __restrict__ stdv, float* __restrict__ rmean, float* __restrict__ rvar) {
    FIN_CHANNEL();
    const float var = part_sum(part, nblk, C, c, 0, lane) / (float)R;
    if (lane != 0 || !cown) return;
    stdv[c] = sqrtf(var + 1e-5f);
    rmean[c] = rmean[c] * 0.9f + mean[c] * 0.1f;
    rvar[c] = rvar[c] * 0.9f + var * 0.1f;
}

// BN backward sums: dbeta[c] = sum dz, dgamma[c] = sum dz*yhat
// slot (sharded batch): also this rank's exchange slot [dbeta | dgamma] (two copies fewer per BN)
__global__ void finalize_bnback_kernel(const float* __restrict__ part, int nblk, int C, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float* __restrict__ slot = nullptr) {
    FIN_CHANNEL();
    float bg[2];
    part_sums<2>(part, nblk, C, c, {0, 1}, lane, bg);
    const float b = bg[0], g = bg[1];
    if (lane == 0 && cown) {
        dbeta[c] = b;
        dgamma[c] = g;
        if (slot) {
            slot[c] = b;
            slot[C + c] = g;
        }
    }
}
// BN forward statistics from per-board partials (BoardStats, STATS 1): mean = sum / R, and the
// squared deviations combined as sum_b [M2_b + 64 (mean_b - mean)^2] (Chan, Golub & LeVeque's
// pairwise update, every board 64 rows); then as finalize_var_kernel.  Fixed order per channel.
__global__ void bn_board_var_kernel(const float* __restrict__ part, int nb, int C, int R, float* __restrict__ mean,
                                    float* __restrict__ stdv, float* __restrict__ rmean, float* __restrict__ rvar) {
    FIN_CHANNEL();
    float s, m2;
    board_stats(part, nb, C, c, R, lane, s, m2);
    const float mu = s / (float)R;
    if (lane != 0 || !cown) return;
    const float var = m2 / (float)R;
    mean[c] = mu;
    stdv[c] = sqrtf(var + 1e-5f);
    rmean[c] = rmean[c] * 0.9f + mu * 0.1f;
    rvar[c] = rvar[c] * 0.9f + var * 0.1f;
}
// Sharded batch (az_trainer_set_sharded): one global batch split over the ranks, BatchNorm
// statistics over all of it (burn BatchNorm on the reference's single 512 batch, agent.rs:37,41,
// training.rs:159).  Each rank writes its slot of a [world][2 slot + 1] exchange buffer -- the sum
// S[c] of its rows, the squared deviations M2[c] from its OWN mean, and its row count n -- the
// buffer (zero outside the slot) is summed over ranks (an all-gather through the sum all-reduce,
// exact: x + 0 = x), and bn_global_kernel combines the slots in rank order with Chan et al.'s
// pairwise update.  At world = 1 every value is bit-identical to bn_board_var_kernel /
// finalize_var_kernel: S / n is the same division, the rank's deviation term is exactly 0.
// bn_local_kernel: the slot from per-board partials (BoardStats STATS 1), the arithmetic of
// bn_board_var_kernel up to its mean and m2.
__global__ void bn_local_kernel(const float* __restrict__ part, int nb, int C, int R, float* __restrict__ slot,
                                int sstride) {
    FIN_CHANNEL();
    float s, m2;
    board_stats(part, nb, C, c, R, lane, s, m2);
    if (lane != 0 || !cown) return;
    slot[c] = s;
    slot[sstride + c] = m2;
    if (c == 0) slot[2 * sstride] = (float)R;
}
__global__ void set_value_kernel(float* __restrict__ p, float v) { *p = v; }
// out[i] = sum over ranks r = 0, 1, ... (in order) of slots[r stride + i]
__global__ void sum_slots_kernel(const float* __restrict__ slots, int world, size_t stride, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = slots[i];
    for (int r = 1; r < world; r++) s += slots[(size_t)r * stride + i];
    out[i] = s;
}
// the ranks' slots -> batch mean / std and the running statistics (momentum 0.1, as
// finalize_var_kernel); nglob (BN 0 only): the global row count for the loss and the BN backward
// coff: the BatchNorm's first channel in the slots (the two head BatchNorms share one exchange)
__global__ void bn_global_kernel(const float* __restrict__ xb, int world, int C, int sstride, int coff,
                                 float* __restrict__ mean, float* __restrict__ stdv, float* __restrict__ rmean,
                                 float* __restrict__ rvar, float* __restrict__ nglob) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const size_t rs = 2 * (size_t)sstride + 1;
    float n = 0.0f, s = 0.0f;
    for (int r = 0; r < world; r++) {
        n += xb[r * rs + 2 * sstride];
        s += xb[r * rs + coff + c];
    }
    const float mu = s / n;
    float m2 = 0.0f;
    for (int r = 0; r < world; r++) {
        const float nr = xb[r * rs + 2 * sstride];
        if (nr == 0.0f) continue;
        const float d = xb[r * rs + coff + c] / nr - mu;
        m2 += xb[r * rs + sstride + coff + c] + nr * (d * d);
    }
    const float var = m2 / n;
    mean[c] = mu;
    stdv[c] = sqrtf(var + 1e-5f);
    rmean[c] = rmean[c] * 0.9f + mu * 0.1f;
    rvar[c] = rvar[c] * 0.9f + var * 0.1f;
    if (c == 0 && nglob) *nglob = n;
}
#undef FIN_CHANNEL

// column sums (16-byte loads when the channel layout allows it, else the scalar kernel), then the
// finalize kernel of `fin`.  (Finalizing in the last row block to arrive instead -- an arrival
// counter and device-scope fences -- measured 6.4 -> 38.7 us for the MODE 0 sums: each block's
// release fence writes back its XCD's L2, dirty with the previous kernel's output.)
template <int MODE>
void launch_colsum(dim3 g, hipStream_t st, const float* V, int ld, int C, int R, const float* mean, const float* stdv,
                   const float* O, const float* Y, float* part, const ColFin& fin) {
    const bool vec = C % 4 == 0 && ld % 4 == 0 && ((uintptr_t)V & 15) == 0 && (!O || ((uintptr_t)O & 15) == 0) &&
                     (!Y || ((uintptr_t)Y & 15) == 0);
    if (vec) colsum4_kernel<MODE><<<g, 256, 0, st>>>(V, ld, C, R, mean, stdv, O, Y, part);
    else colsum_kernel<MODE><<<g, 256, 0, st>>>(V, ld, C, R, mean, stdv, O, Y, part);
    const int nb = (int)g.x, fg = finalize_grid(C);
    if (fin.kind == FIN_SUM) finalize_sum_kernel<<<fg, FIN_THREADS, 0, st>>>(part, nb, C, fin.a);
    else if (fin.kind == FIN_MEAN) finalize_mean_kernel<<<fg, FIN_THREADS, 0, st>>>(part, nb, C, R, fin.a);
    else if (fin.kind == FIN_VAR) finalize_var_kernel<<<fg, FIN_THREADS, 0, st>>>(part, nb, C, R, fin.mean, fin.a, fin.b, fin.c);
    else finalize_bnback_kernel<<<fg, FIN_THREADS, 0, st>>>(part, nb, C, fin.a, fin.b);
}

// ------------------------------------------------------------------ element-wise
// out = relu(((y - mean) / std) * gamma + beta [+ res])   (burn BatchNorm::forward_shared + relu)
__global__ void bn_apply_kernel(const float* __restrict__ Y, int ld, int C, int R, const float* __restrict__ mean,
                                const float* __restrict__ stdv, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ res, float* __restrict__ out) {
    const size_t n = (size_t)R * C;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(e / C), c = (int)(e % C);
        const size_t o = (size_t)r * ld + c;
        float v = ((Y[o] - mean[c]) / stdv[c]) * gamma[c] + beta[c];
        if (res) v += res[o];
        out[o] = fmaxf(v, 0.0f);
    }
}

// The same four channels per thread (16-byte accesses; C a power of two in [4, 1024], ld and
// the pointers 16-byte multiples): thread t owns channel quad t % (C / 4) -- its parameters are
// loaded once -- and rows t / (C / 4) + k (256 / (C / 4)), so no per-element index division (the
// scalar kernel: 16.2 us at 32768 x 256)
__global__ void __launch_bounds__(256) bn_apply4_kernel(const float* __restrict__ Y, int ld, int C, int R,
                                                        const float* __restrict__ mean, const float* __restrict__ stdv,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        const float* __restrict__ res, float* __restrict__ out) {
    const int cq = C / 4, c = 4 * (threadIdx.x % cq), rs = 256 / cq;
    const float4 mu = *reinterpret_cast<const float4*>(mean + c), sd = *reinterpret_cast<const float4*>(stdv + c);
    const float4 ga = *reinterpret_cast<const float4*>(gamma + c), be = *reinterpret_cast<const float4*>(beta + c);
    for (int r = blockIdx.x * rs + (int)threadIdx.x / cq; r < R; r += gridDim.x * rs) {
        const size_t o = (size_t)r * ld + c;
        const float4 y = *reinterpret_cast<const float4*>(Y + o);
        float4 v = make_float4(((y.x - mu.x) / sd.x) * ga.x + be.x, ((y.y - mu.y) / sd.y) * ga.y + be.y,
                               ((y.z - mu.z) / sd.z) * ga.z + be.z, ((y.w - mu.w) / sd.w) * ga.w + be.w);
        if (res) {
            const float4 q = *reinterpret_cast<const float4*>(res + o);
            v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
        }
        *reinterpret_cast<float4*>(out + o) =
            make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
    }
}

// BN backward: dy = (gamma/std) * (dz - dbeta/R - yhat*dgamma/R), dz = dout*(o > 0);
// if dres: dres = dz (the residual branch's gradient, added by the next data-grad GEMM)
__global__ void bn_back_kernel(const float* __restrict__ dout, const float* __restrict__ O, const float* __restrict__ Y,
                               int ld, int C, int R, const float* __restrict__ mean, const float* __restrict__ stdv,
                               const float* __restrict__ gamma, const float* __restrict__ dgamma,
                               const float* __restrict__ dbeta, float* __restrict__ dy, float* __restrict__ dres,
                               const float* __restrict__ nglob) {
    const size_t n = (size_t)R * C;
    const float invR = 1.0f / (nglob ? nglob[vgpr_index(0)] : (float)R);
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(e / C), c = (int)(e % C);
        const size_t o = (size_t)r * ld + c;
        const float dz = O[o] > 0.0f ? dout[o] : 0.0f;
        const float yhat = (Y[o] - mean[c]) / stdv[c];
        dy[o] = (gamma[c] / stdv[c]) * (dz - dbeta[c] * invR - yhat * dgamma[c] * invR);
        if (dres) dres[o] = dz;
    }
}

// bn_back_kernel four channels per thread, laid out as bn_apply4_kernel
__global__ void __launch_bounds__(256) bn_back4_kernel(const float* __restrict__ dout, const float* __restrict__ O,
                                                       const float* __restrict__ Y, int ld, int C, int R,
                                                       const float* __restrict__ mean, const float* __restrict__ stdv,
                                                       const float* __restrict__ gamma, const float* __restrict__ dgamma,
                                                       const float* __restrict__ dbeta, float* __restrict__ dy,
                                                       float* __restrict__ dres, float* __restrict__ bsum,
                                                       const float* __restrict__ nglob) {
    const int cq = C / 4, c = 4 * (threadIdx.x % cq), rs = 256 / cq;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);   // bsum: this thread's rows of dy, in order
    const float invR = 1.0f / (nglob ? nglob[vgpr_index(0)] : (float)R);   // sharded batch: all ranks' rows (vector load)
    const float4 mu = *reinterpret_cast<const float4*>(mean + c), sd = *reinterpret_cast<const float4*>(stdv + c);
    const float4 ga = *reinterpret_cast<const float4*>(gamma + c), dg = *reinterpret_cast<const float4*>(dgamma + c);
    const float4 db = *reinterpret_cast<const float4*>(dbeta + c);
    for (int r = blockIdx.x * rs + (int)threadIdx.x / cq; r < R; r += gridDim.x * rs) {
        const size_t o = (size_t)r * ld + c;
        const float4 d = *reinterpret_cast<const float4*>(dout + o), ov = *reinterpret_cast<const float4*>(O + o);
        const float4 y = *reinterpret_cast<const float4*>(Y + o);
        const float4 dz = make_float4(ov.x > 0.0f ? d.x : 0.0f, ov.y > 0.0f ? d.y : 0.0f, ov.z > 0.0f ? d.z : 0.0f,
                                      ov.w > 0.0f ? d.w : 0.0f);
        const float4 d4 = make_float4((ga.x / sd.x) * (dz.x - db.x * invR - ((y.x - mu.x) / sd.x) * dg.x * invR),
                                      (ga.y / sd.y) * (dz.y - db.y * invR - ((y.y - mu.y) / sd.y) * dg.y * invR),
                                      (ga.z / sd.z) * (dz.z - db.z * invR - ((y.z - mu.z) / sd.z) * dg.z * invR),
                                      (ga.w / sd.w) * (dz.w - db.w * invR - ((y.w - mu.w) / sd.w) * dg.w * invR));
        *reinterpret_cast<float4*>(dy + o) = d4;
        if (dres) *reinterpret_cast<float4*>(dres + o) = dz;
        acc.x += d4.x; acc.y += d4.y; acc.z += d4.z; acc.w += d4.w;
    }
    // the conv bias gradient (sum of dy over rows) as per-workgroup partials in the column-sum
    // layout part[block][2][C] (finalize_sum_kernel), instead of another pass over dy
    if (bsum) {
        __shared__ float4 red[256];
        red[threadIdx.x] = acc;
        __syncthreads();
        if ((int)threadIdx.x < cq) {
            float4 a = red[threadIdx.x];
            for (int k = 1; k < rs; k++) {
                const float4 b = red[k * cq + threadIdx.x];
                a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
            }
            *reinterpret_cast<float4*>(bsum + (size_t)blockIdx.x * 2 * C + c) = a;
        }
    }
}

// planes [B][19][64] (to_tensor layout, chess.rs:191-245) -> X0 [B*64][X0C] (channels >= 19 zero;
// X0C = 32, the smallest multiple of the convs' 16-channel K chunk: the input conv ran on 64 padded
// channels before round 4, 3.4x the 19 real ones -- 96 -> 56 us per step.  Its weight grad keeps its
// 64-wide k tile (skipping the empty half with a uniform branch around the MFMAs measured slower,
// and slowed the 1-tap instantiation 2x))
constexpr int X0C = 32;
__global__ void planes_kernel(const float* __restrict__ planes, int B, float* __restrict__ x0) {
    const size_t n = (size_t)B * 64 * X0C;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(e % X0C), r = (int)(e / X0C), b = r >> 6, s = r & 63;
        x0[e] = c < 19 ? planes[((size_t)b * 19 + c) * 64 + s] : 0.0f;
    }
}

// value-head flatten (agent.rs:135: reshape [B, 8*8*8], index c*64 + s) and its inverse
__global__ void vflat_kernel(float* __restrict__ a40, float* __restrict__ vflat, int B, int inverse) {
    const size_t n = (size_t)B * 512;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(e / 512), i = (int)(e % 512), c = i >> 6, s = i & 63;
        const size_t o = ((size_t)b * 64 + s) * 64 + 32 + c;
        if (inverse) a40[o] = vflat[e];
        else vflat[e] = a40[o];
    }
}

// ------------------------------------------------------------------ loss (training.rs:277-292)
// One 256-thread block per board.  Policy: p = softmax(logits) over the 4096 flat entries
// (index c*64 + s, agent.rs:126-129), loss_b = -sum t*log(p + 1e-5); dlogit = p*(G - sum p*G),
// G = -t/(p + 1e-5)/B.  Value: v = tanh(relu(h1) . w2 + b2), loss_b = (v - z)^2,
// dlogit_v = 0.5*2*(v - z)/B * (1 - v^2); dh1 = dlogit_v * w2 * (h1 > 0).
// Per-board outputs: loss[b] = {policy, value}; vpart[b] = {dW2[64], db2}.
__global__ void __launch_bounds__(256)
loss_kernel(const float* __restrict__ logits, const float* __restrict__ tpol, const float* __restrict__ h1,
            const float* __restrict__ tval, const float* __restrict__ w2, const float* __restrict__ b2, int B,
            float* __restrict__ dlogits, float* __restrict__ dh1, float* __restrict__ loss,
            float* __restrict__ vpart, const float* __restrict__ nglob) {
    __shared__ float red[256];
    __shared__ float bc[4];
    const int b = blockIdx.x, t = threadIdx.x;
    const float* L = logits + (size_t)b * 64 * 64;
    const float* T = tpol + (size_t)b * 4096;
    float l[16];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int i = t + 256 * j;
        l[j] = L[(i & 63) * 64 + (i >> 6)];
        mx = fmaxf(mx, l[j]);
    }
    auto block_reduce = [&](float v, bool is_max) -> float {
        red[t] = v;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (t < o) red[t] = is_max ? fmaxf(red[t], red[t + o]) : red[t] + red[t + o];
            __syncthreads();
        }
        const float r = red[0];
        __syncthreads();
        return r;
    };
    mx = block_reduce(mx, true);
    float se = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; j++) { l[j] = expf(l[j] - mx); se += l[j]; }
    se = block_reduce(se, false);
    const float invB = 1.0f / (nglob ? nglob[vgpr_index(0)] / 64.0f : (float)B);   // sharded: the global batch (vector load)
    float lp = 0.0f, pg = 0.0f, G[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int i = t + 256 * j;
        const float p = l[j] / se, q = T[i];
        l[j] = p;
        lp += q * logf(p + 1e-5f);
        G[j] = -q / (p + 1e-5f) * invB;
        pg += p * G[j];
    }
    lp = block_reduce(lp, false);
    pg = block_reduce(pg, false);
    float* D = dlogits + (size_t)b * 64 * 64;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int i = t + 256 * j;
        D[(i & 63) * 64 + (i >> 6)] = l[j] * (G[j] - pg);
    }
    // value tail
    const float hv = t < 64 ? h1[(size_t)b * 64 + t] : 0.0f;
    const float a = fmaxf(hv, 0.0f);
    const float dot = block_reduce(t < 64 ? a * w2[t] : 0.0f, false);
    if (t == 0) {
        const float v = tanhf(dot + b2[0]);
        const float d = v - tval[b];
        bc[0] = d * 2.0f * 0.5f * invB * (1.0f - v * v);
        loss[b * 2 + 0] = -lp;
        loss[b * 2 + 1] = d * d;
    }
    __syncthreads();
    const float dl = bc[0];
    if (t < 64) {
        dh1[(size_t)b * 64 + t] = hv > 0.0f ? dl * w2[t] : 0.0f;
        vpart[(size_t)b * 65 + t] = dl * a;
    }
    if (t == 0) vpart[(size_t)b * 65 + 64] = dl;
}

// ------------------------------------------------------------------ weight repacking
// conv [co][ci][3][3] (burn) -> Wf[t][k][co] (k < kpad, rows >= cin zero) and Wd[t][co][ci] = Wf[8-t]^T
// ------------------------------------------------------------------ Winograd forward / data grad
// The 3x3 F -> F convs of the residual tower (F = 256) as Winograd F(2x2, 3x3) -- the inference
// tower's core (wino.h), 2.25x fewer MFMAs than the implicit GEMM, f32 throughout -- one board at
// a time per 512-thread workgroup: the board's 64 rows of X into LDS, wino_core, Y (+ addend) back
// to HBM with no ReLU (BatchNorm runs in training mode after it).  Persistent: AZ_TRAIN_WG
// workgroups (one per CU) loop over the boards, the weight ring carrying the conv's first steps
// into the next board (round 5: data-grad convs -2..4 us, bit-identical; the one-board-per-
// workgroup grid left a re-dispatch gap of up to 5 us per CU between its two boards).  The data grad is the same conv of
// dY with the flipped, transposed kernel (U built by wino_weights_kernel with flip = 1).
// STATS: per-board BatchNorm statistics of the output from the epilogue, into part[board][2][F]
// (the layout of the column-sum partials, one "row block" per board):
//   1 (forward, the output is the BN input): sum and sum of squared deviations from the board's
//     own mean -- combined over boards by bn_board_var_kernel (Chan et al.'s pairwise update);
//   2 (data grad, the output is the BN backward's dout): sum dz and sum dz * yhat with
//     dz = dout * (O > 0), yhat = (Ybn - mean) / std -- summed over boards by finalize_bnback_kernel.
// Either replaces two passes over the 32 MB output (colsum4 + finalize twice, or colsum4<2>).
#ifndef AZ_TRAIN_WG
#define AZ_TRAIN_WG 256   // persistent Winograd-conv workgroups: one per CU of MI355X
#endif
struct BoardStats {
    float* part;
    const float* O;      // STATS 2: the BN's ReLU output
    const float* Ybn;    // STATS 2: the BN's input
    const float* mean;   // STATS 2
    const float* stdv;   // STATS 2
    const float *gamma, *beta;   // STATS 2 with ORC & 2: O's sign recomputed from Ybn (no residual)
};
// BNIN: the conv's input is the BatchNorm + ReLU (+ residual) of the previous conv's output,
// applied while the board's rows are staged (bn_apply4_kernel's arithmetic, element for element),
// and written out as the saved activation the backward needs -- the separate bn_apply pass over
// the 32 MB layer (a read of Y and the residual, a write, and the conv's re-read) is gone.
struct BnIn {
    const float *mean, *stdv, *gamma, *beta;
    const float* res;    // the block input added before the ReLU (BN2), or null (BN0 / BN1)
    float* out;          // relu(bn(X) [+ res]): hh[b] or xs[b]
};
// XIN 2 (data-grad convs): the conv's input dy is the BatchNorm backward of X = dout (the ReLU
// output's gradient), computed while the board's rows are staged (bn_back4_kernel's arithmetic,
// element for element) and written out for the weight grad; dres (BN2) gets dz; bsum gets the
// board's sum of dy per channel (the producing conv's bias gradient, summed over boards later)
struct BnBack {
    const float *O, *Y, *mean, *stdv, *gamma, *dgamma, *dbeta, *nglob;
    float *dy, *dres, *bsum;
    int R;
    const float* beta;   // ORC & 1: O's sign recomputed from Y (no residual)
};
// ORC (round 6): a BatchNorm with no residual (BN 0 and every block's BN1) has O = relu(v) with
// v = ((Y - mean) / std) * gamma + beta, the exact float expression the forward evaluated (BnIn staging
// or bn_apply4_kernel, -ffp-contract=off), so O > 0 <=> v > 0 and the backward need not read O:
// bit 0 -- the BN backward in the staging (BnBack), bit 1 -- the STATS 2 epilogue (BoardStats).
// Each drops one of the three 64 KB-per-board streams of its phase (the staging and the epilogue
// are bound by HBM bandwidth: every CU runs them at the same moment).
__device__ __forceinline__ bool relu_pos(float y, float mu, float sd, float ga, float be) {
    return ((y - mu) / sd) * ga + be > 0.0f;
}
__device__ __forceinline__ f32x4 sum16(f32x4 v) {   // over the 16 lanes of a row (fixed butterfly)
#pragma unroll
    for (int m = 1; m < 16; m <<= 1)
#pragma unroll
        for (int r = 0; r < 4; r++) v[r] += __shfl_xor(v[r], m, 64);
    return v;
}
template <bool ADD, int STATS, int XIN, int ORC = 0>
__global__ void __launch_bounds__(512)
conv_wino_train_kernel(const float* __restrict__ X, const uint4* __restrict__ U, unsigned ubytes,
                       const float* __restrict__ bias, const float* __restrict__ addend, float* __restrict__ Y,
                       BoardStats bs, BnIn bn, BnBack bb, int nboards, unsigned long long* trb) {
    constexpr int F = 256, NN = WinoCfg<F>::NN, XSn = WinoCfg<F>::XS, PF = WinoCfg<F>::PF, RS = F / 4 + 2;
    constexpr int XSZ = 64 * RS, VSZ = 2 * WinoCfg<F>::CH * 1024 / 16, PAD = WINO_PAD_SQ * RS;
    __shared__ __attribute__((aligned(16))) uint4 lds[PAD + XSZ + PAD + VSZ];
    uint4* act = lds + PAD;                              // zero squares either side (wino_core)
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int c = tid; c < PAD; c += 512) {
        lds[c] = make_uint4(0, 0, 0, 0);
        act[XSZ + c] = make_uint4(0, 0, 0, 0);
    }
    // persistent: the workgroup loops over boards blockIdx.x, + gridDim.x, ...; the weight ring's
    // refills past the conv's last step read its first steps again (rN = rW), for the next board
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)U, (short)0, (int)ubytes, 0x00020000);
    const int voff = wino_voff<F>(w, lane);
    f32x4 wr[PF][XSn][NN];
#pragma unroll
    for (int i = 0; i < PF; i++)
#pragma unroll
        for (int xs = 0; xs < XSn; xs++)
#pragma unroll
            for (int n = 0; n < NN; n++)
                wr[i][xs][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                             rW, voff + n * 1024 + wino_toff<F>(0, i * XSn + xs), 0, 0));
#pragma unroll 1
    for (int bid = blockIdx.x; bid < nboards; bid += gridDim.x) {
        const size_t row0 = (size_t)vgpr_index(bid) * 64;
        const uint4* X4 = reinterpret_cast<const uint4*>(X) + row0 * (F / 4);
        unsigned long long* const tr = trb && w == 0 ? trb + (size_t)vgpr_index(bid) * 8 : nullptr;
        wino_stamp(tr, 0);
#ifdef AZ_TOWER_TRACE
        if (tr && lane == 0) {   // where the board ran: HW_ID (CU, SIMD, SE ...) and XCC_ID
            tr[4] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
            tr[5] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));
        }
#endif
        // (Round 6: the next board's XIN 1 staging beside this board's MFMAs -- one float4 per thread
        // per input chunk, after that chunk's transform, through a per-step hook in wino_core --
        // was bit-identical and measured 21.26 vs 21.15 ms per step: the BatchNorm apply's IEEE
        // divisions cost the MFMA waves more than the staging phase they replaced, and only every
        // second board's staging can move.  profiles/r06w_ab_prestage_b512.txt; not kept.)
        if constexpr (XIN == 1) {   // thread = channel quad tid % 64 (F / 4 = 64 divides 512) x rows tid / 64 + 8 k
            static_assert(F / 4 == 64, "BNIN staging assumes 64 channel quads");
            const int cq = tid & 63;
            const float4 mu = reinterpret_cast<const float4*>(bn.mean)[cq], sd = reinterpret_cast<const float4*>(bn.stdv)[cq];
            const float4 ga = reinterpret_cast<const float4*>(bn.gamma)[cq], be = reinterpret_cast<const float4*>(bn.beta)[cq];
            const float4* R4 = bn.res ? reinterpret_cast<const float4*>(bn.res) + row0 * (F / 4) : nullptr;
            float4* O4 = reinterpret_cast<float4*>(bn.out) + row0 * (F / 4);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int c = tid + 512 * k;
                const float4 y = reinterpret_cast<const float4*>(X4)[c];
                float4 v = make_float4(((y.x - mu.x) / sd.x) * ga.x + be.x, ((y.y - mu.y) / sd.y) * ga.y + be.y,
                                       ((y.z - mu.z) / sd.z) * ga.z + be.z, ((y.w - mu.w) / sd.w) * ga.w + be.w);
                if (R4) {
                    const float4 q = R4[c];
                    v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
                }
                const float4 o = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
                O4[c] = o;
                act[(c / (F / 4)) * RS + cq] = __builtin_bit_cast(uint4, o);
            }
        } else if constexpr (XIN == 2) {   // the same thread layout; X = dout
            static_assert(F / 4 == 64, "BnBack staging assumes 64 channel quads");
            const int cq = tid & 63;
            const float invR = 1.0f / (bb.nglob ? bb.nglob[vgpr_index(0)] : (float)bb.R);   // (a vector load: written by an earlier launch)
            const float4 mu = reinterpret_cast<const float4*>(bb.mean)[cq], sd = reinterpret_cast<const float4*>(bb.stdv)[cq];
            const float4 ga = reinterpret_cast<const float4*>(bb.gamma)[cq], dg = reinterpret_cast<const float4*>(bb.dgamma)[cq];
            const float4 db = reinterpret_cast<const float4*>(bb.dbeta)[cq];
            float4 be = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr ((ORC & 1) != 0) be = reinterpret_cast<const float4*>(bb.beta)[cq];
            const size_t o0 = row0 * (F / 4);
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const size_t c = o0 + tid + 512 * k;
                const float4 d = reinterpret_cast<const float4*>(X)[c];
                const float4 y = reinterpret_cast<const float4*>(bb.Y)[c];
                bool px, py, pz, pw;   // O > 0
                if constexpr ((ORC & 1) != 0) {
                    px = relu_pos(y.x, mu.x, sd.x, ga.x, be.x); py = relu_pos(y.y, mu.y, sd.y, ga.y, be.y);
                    pz = relu_pos(y.z, mu.z, sd.z, ga.z, be.z); pw = relu_pos(y.w, mu.w, sd.w, ga.w, be.w);
                } else {
                    const float4 ov = reinterpret_cast<const float4*>(bb.O)[c];
                    px = ov.x > 0.0f; py = ov.y > 0.0f; pz = ov.z > 0.0f; pw = ov.w > 0.0f;
                }
                const float4 dz = make_float4(px ? d.x : 0.0f, py ? d.y : 0.0f, pz ? d.z : 0.0f, pw ? d.w : 0.0f);
                const float4 d4 = make_float4((ga.x / sd.x) * (dz.x - db.x * invR - ((y.x - mu.x) / sd.x) * dg.x * invR),
                                              (ga.y / sd.y) * (dz.y - db.y * invR - ((y.y - mu.y) / sd.y) * dg.y * invR),
                                              (ga.z / sd.z) * (dz.z - db.z * invR - ((y.z - mu.z) / sd.z) * dg.z * invR),
                                              (ga.w / sd.w) * (dz.w - db.w * invR - ((y.w - mu.w) / sd.w) * dg.w * invR));
                reinterpret_cast<float4*>(bb.dy)[c] = d4;
                if (bb.dres) reinterpret_cast<float4*>(bb.dres)[c] = dz;
                act[(tid + 512 * k) / (F / 4) * RS + cq] = __builtin_bit_cast(uint4, d4);
                acc.x += d4.x; acc.y += d4.y; acc.z += d4.z; acc.w += d4.w;
            }
            // the board's bias partial: the 8 row phases of each channel quad, in order, through the
            // (not yet written) V buffers
            float4* red = reinterpret_cast<float4*>(lds + PAD + XSZ + PAD);
            red[tid] = acc;
            __syncthreads();
            if (tid < 64) {
                float4 a = red[tid];
                for (int k = 1; k < 8; k++) {
                    const float4 q = red[64 * k + tid];
                    a.x += q.x; a.y += q.y; a.z += q.z; a.w += q.w;
                }
                reinterpret_cast<float4*>(bb.bsum + (size_t)vgpr_index(bid) * 2 * F)[tid] = a;   // [board][2][F]
            }
        } else {
            for (int c = tid; c < 64 * (F / 4); c += 512) act[(c / (F / 4)) * RS + c % (F / 4)] = X4[c];
        }
        __syncthreads();   // (XIN 2: also orders the bias partial's reads of V before wino_core writes V)
        wino_stamp(tr, 1);
        f32x4 y[NN][4];
        wino_core<F>(reinterpret_cast<char*>(act), (XSZ + PAD) * 16, rW, rW, bias, wr, w, lane, y);
        wino_stamp(tr, 2);
        const int l16 = lane & 15, h = lane >> 4, ty = l16 >> 2, tx = l16 & 3;
        const int co0 = w * 16 * NN + h * 4;
        f32x4 s0[NN], s1[NN];
#pragma unroll
        for (int n = 0; n < NN; n++) {
            s0[n] = f32x4{0.f, 0.f, 0.f, 0.f};
            s1[n] = s0[n];
            f32x4 mu = s0[n], sd = s0[n], ga = s0[n], be = s0[n];
            if constexpr (STATS == 2) {
                mu = *reinterpret_cast<const f32x4*>(bs.mean + co0 + n * 16);
                sd = *reinterpret_cast<const f32x4*>(bs.stdv + co0 + n * 16);
                if constexpr ((ORC & 2) != 0) {
                    ga = *reinterpret_cast<const f32x4*>(bs.gamma + co0 + n * 16);
                    be = *reinterpret_cast<const f32x4*>(bs.beta + co0 + n * 16);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const size_t o = (row0 + (2 * ty + (q >> 1)) * 8 + 2 * tx + (q & 1)) * F + co0 + n * 16;
                f32x4 v = y[n][q];
                if constexpr (ADD) v += *reinterpret_cast<const f32x4*>(addend + o);
                *reinterpret_cast<f32x4*>(Y + o) = v;
                if constexpr (STATS == 1) {
                    y[n][q] = v;
                    s0[n] += v;
                } else if constexpr (STATS == 2) {
                    f32x4 ov = s0[n];
                    if constexpr ((ORC & 2) == 0) ov = *reinterpret_cast<const f32x4*>(bs.O + o);
                    const f32x4 yb = *reinterpret_cast<const f32x4*>(bs.Ybn + o);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const bool pos = (ORC & 2) != 0 ? relu_pos(yb[r], mu[r], sd[r], ga[r], be[r]) : ov[r] > 0.0f;
                        const float dz = pos ? v[r] : 0.0f;
                        s0[n][r] += dz;
                        s1[n][r] += dz * ((yb[r] - mu[r]) / sd[r]);
                    }
                }
            }
        }
        if constexpr (STATS != 0) {
#pragma unroll
            for (int n = 0; n < NN; n++) {
                s0[n] = sum16(s0[n]);
                if constexpr (STATS == 1) {
                    const f32x4 mb = s0[n] / 64.0f;   // the board's mean (64 squares)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const f32x4 d = y[n][q] - mb;
                        s1[n] += d * d;
                    }
                }
                s1[n] = sum16(s1[n]);
                if (l16 == 0) {
                    float* pb = bs.part + (size_t)vgpr_index(bid) * 2 * F + co0 + n * 16;
                    *reinterpret_cast<f32x4*>(pb) = s0[n];
                    *reinterpret_cast<f32x4*>(pb + F) = s1[n];
                }
            }
        }
        wino_stamp(tr, 3);
        // every wave is done with ACT and V before the next board's staging.  (Round 6: without
        // this barrier -- legal: the staging writes only ACT and V buffer 0, both dead since the
        // last chunk's barrier -- a done wave would stage beside the others' epilogues; measured
        // flat, 22.00-22.10 vs 21.99-22.02 ms per step, profiles/r06d_ab_endbar.txt.)
        __syncthreads();
    }
}

// ---------------------------------------------------------------- two workgroups per CU
// conv_wino_half_kernel: conv_wino_train_kernel's conv, staging and statistics, bit for bit, by two
// workgroups per board that own half of the output channels each and stream the input through
// LDS in 16-channel chunks instead of holding the whole board (52 KB of LDS, 4 waves): two
// workgroups share a CU, so one's staging loads, barriers, epilogue and launch gap run beside the
// other's MFMAs.  (Phase stamps of the one-board kernel, tools/train_trace.py on MI355X: staging +
// epilogue + the gap between a CU's boards were 13 % of the forward conv's time and 27 % of the
// data-grad conv's, with the MFMA core at 88 % of its issue bound.)
// The price: both halves transform the whole input (a few % of VALU beside the MFMAs) and read it
// (the second read an L2 hit when the halves run together: both halves of a board go to one XCD).
// Per chunk k (16 channels, 16 ring steps): the transform of chunk k + 1 (ACT slot (k + 1) & 1 ->
// V[(k + 1) & 1]) early in the chunk, the staging of chunk k + 2 (global loads at the first step,
// BatchNorm arithmetic + slot write at the last) into the slot chunk k left, one barrier.
#ifndef AZ_PART_PF
#define AZ_PART_PF 8      // ring prefetch steps of the quarter-channel kernel (one 16-channel block per wave)
#endif
#ifndef AZ_HALF_ISSUE
#define AZ_HALF_ISSUE 0   // staging loads of chunk k + 2 at chunk k's first step (1: of chunk k + 3 at its last)
#endif
namespace hk {
constexpr int F = 256, CH = 16, NCH = F / CH, NWV = 4, PF = 2, SPX = 16, LA = 4, TSPLIT = 2;
constexpr int RS = CH / 4 + 2;                 // uint4 per square in a slot (+2: the patch reads' banks)
constexpr int R16 = RS * 16, ROW = 8 * R16;    // bytes per square, per board row
constexpr int SLOT = 64 * RS, PADU = 8 * RS;   // uint4: one chunk of the board, one zero row
constexpr int XST = CH * 64, VBYTES = CH * 1024;
constexpr int SLOTS = 3 * PADU + 2 * SLOT;     // [zero row][slot 0][zero row][slot 1][zero row]
constexpr int PAR = 5 * F / 4;                 // uint4: the staging's per-channel parameters
constexpr int VB0 = (SLOTS + PAR) * 16;        // bytes: V[2]
constexpr int LDS_U4 = SLOTS + PAR + 2 * VBYTES / 16;
__device__ __forceinline__ int slot_off(int s) { return (PADU + s * (SLOT + PADU)) * 16; }
}  // namespace hk

// one float4 (4 channels of one square) of chunk k per thread: quad tid & 3, square tid >> 2
template <int XIN> struct HalfStage {
    float4 a, b, c;
    size_t e;
    __device__ __forceinline__ void issue(const float* X, const BnIn& bn, const BnBack& bb, size_t row0, int tid, int k) {
        e = (row0 + (tid >> 2)) * (hk::F / 4) + 4 * k + (tid & 3);
        a = reinterpret_cast<const float4*>(X)[e];
        if constexpr (XIN == 1) {
            if (bn.res) b = reinterpret_cast<const float4*>(bn.res)[e];
        } else if constexpr (XIN == 2) {
            b = reinterpret_cast<const float4*>(bb.O)[e];
            c = reinterpret_cast<const float4*>(bb.Y)[e];
        }
    }
    // the arithmetic of conv_wino_train_kernel's staging, element for element; the owner of the
    // chunk writes the activation / dy / dres
    __device__ __forceinline__ void finish(char* l, const BnIn& bn, const BnBack& bb, float invR, int tid, int k, int s,
                                           bool owner) const {
        const int cq = 4 * k + (tid & 3);
        const float4* par = reinterpret_cast<const float4*>(l + hk::SLOTS * 16);
        float4 v = a;
        if constexpr (XIN == 1) {
            const float4 mu = par[cq], sd = par[64 + cq], ga = par[128 + cq], be = par[192 + cq];
            const float4 y = a;
            v = make_float4(((y.x - mu.x) / sd.x) * ga.x + be.x, ((y.y - mu.y) / sd.y) * ga.y + be.y,
                            ((y.z - mu.z) / sd.z) * ga.z + be.z, ((y.w - mu.w) / sd.w) * ga.w + be.w);
            if (bn.res) {
                v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
            }
            v = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
            if (owner) reinterpret_cast<float4*>(bn.out)[e] = v;
        } else if constexpr (XIN == 2) {
            const float4 mu = par[cq], sd = par[64 + cq], ga = par[128 + cq], dg = par[192 + cq], db = par[256 + cq];
            const float4 d = a, ov = b, y = c;
            const float4 dz = make_float4(ov.x > 0.0f ? d.x : 0.0f, ov.y > 0.0f ? d.y : 0.0f, ov.z > 0.0f ? d.z : 0.0f,
                                          ov.w > 0.0f ? d.w : 0.0f);
            v = make_float4((ga.x / sd.x) * (dz.x - db.x * invR - ((y.x - mu.x) / sd.x) * dg.x * invR),
                            (ga.y / sd.y) * (dz.y - db.y * invR - ((y.y - mu.y) / sd.y) * dg.y * invR),
                            (ga.z / sd.z) * (dz.z - db.z * invR - ((y.z - mu.z) / sd.z) * dg.z * invR),
                            (ga.w / sd.w) * (dz.w - db.w * invR - ((y.w - mu.w) / sd.w) * dg.w * invR));
            if (owner) {
                reinterpret_cast<float4*>(bb.dy)[e] = v;
                if (bb.dres) reinterpret_cast<float4*>(bb.dres)[e] = dz;
            }
        }
        *reinterpret_cast<float4*>(l + hk::slot_off(s) + ((tid >> 2) * hk::RS + (tid & 3)) * 16) = v;
    }
};

// the input transform of one chunk from ACT slot s into V[buf]: WinoXf's item (tile row w, tile
// lane >> 4, channel lane & 15 of the chunk) and arithmetic, over the slot's square stride
struct HalfXf {
    char* l;
    int w, lane;
    __device__ __forceinline__ void load(int s, f32x2 (&d)[4][2]) const {
        const int tl = vgpr_index(lane >> 4);
        const int pc1 = tl * (2 * hk::R16) + (lane & 15) * 4;
        const int pd0 = tl > 0 ? -hk::R16 : 3 * hk::R16, pd3 = tl < 3 ? 2 * hk::R16 : -2 * hk::R16;
        const int b1 = hk::slot_off(s) + pc1 + (2 * w - 1) * hk::ROW;
        const int cb[4] = {b1 + pd0, b1, b1 + hk::R16, b1 + pd3};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const char* p = l + cb[j];
            d[j][0] = f32x2{*reinterpret_cast<const float*>(p), *reinterpret_cast<const float*>(p + hk::ROW)};
            d[j][1] = f32x2{*reinterpret_cast<const float*>(p + 2 * hk::ROW), *reinterpret_cast<const float*>(p + 3 * hk::ROW)};
        }
    }
    __device__ __forceinline__ void store(int buf, const f32x2 (&d)[4][2]) const {
        const int tl = vgpr_index(lane >> 4), tch = lane & 15;
        const f32x2 m = f32x2{tl > 0 ? 1.0f : 0.0f, tl < 3 ? 1.0f : 0.0f};
        f32x2 v[4][2];
        WinoXf<256>::xform(d, m, v);
        char* vb = l + hk::VB0 + buf * hk::VBYTES + (tch >> 2) * 256 +
                   (((4 * w + (lane >> 4)) ^ (2 * ((tch >> 2) & 3))) * 16) + (tch & 3) * 4;
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int rp = 0; rp < 2; rp++) {
                *reinterpret_cast<float*>(vb + ((2 * rp) * 4 + k) * hk::XST) = v[k][rp].x;
                *reinterpret_cast<float*>(vb + ((2 * rp + 1) * 4 + k) * hk::XST) = v[k][rp].y;
            }
    }
};

// XIN 2: the board's sum of dy over its squares for the 16 channels of the chunk in slot s, in
// conv_wino_train_kernel's order (row phases r = 0..7 each over squares r + 8 j, then the phases in
// order); one wave, lane = channel + 16 x phase (r and r + 4)
__device__ __forceinline__ void half_bsum(const char* l, int s, int lane, float* dst) {
    const int ch = lane & 15, r4 = lane >> 4;
    const float* p = reinterpret_cast<const float*>(l + hk::slot_off(s)) + ch;
    float lo = 0.0f, hi = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        lo += p[(r4 + 8 * j) * hk::RS * 4];
        hi += p[(r4 + 4 + 8 * j) * hk::RS * 4];
    }
    float a = lo;
#pragma unroll
    for (int r = 1; r < 8; r++) a += r < 4 ? __shfl(lo, ch + 16 * r, 64) : __shfl(hi, ch + 16 * (r - 4), 64);
    if (lane < 16) dst[ch] = a;
}

// NP = 2 (halves) or 4 (quarters: 256 workgroups at 64 boards, one wave per SIMD of 16 output
// channels, two steps' MFMAs interleaved so that two independent accumulator chains hide the f32
// MFMA's dependent latency; every accumulator still takes its MFMAs in the same order)
template <int NP, bool ADD, int STATS, int XIN>
__global__ void __launch_bounds__(256, 2)
conv_wino_part_kernel(const float* __restrict__ X, const uint4* __restrict__ U, unsigned ubytes,
                      const float* __restrict__ bias, const float* __restrict__ addend, float* __restrict__ Y,
                      BoardStats bs, BnIn bn, BnBack bb, int B, unsigned long long* trb) {
    using namespace hk;
    constexpr int NB = 16 / (NP * NWV);                  // 16-channel output blocks per wave
    constexpr int SPI = NB == 1 ? 2 : 1;                 // ring steps per MFMA group
    // weight-ring prefetch in steps: at NB = 1 a step is 4 MFMAs (128 cycles) of the SIMD's one
    // wave, so 2 steps in flight left every ring wait short of the L2 latency (phase stamps: the
    // core at 33 % of its MFMA bound, profiles/r06ab_trace64.txt).  64-position step: 6.45 / 5.72 /
    // 5.16 / 5.35 ms at 2 / 4 / 8 / 16 steps (profiles/r06ac_*, r06ad_*), bit-identical.  (The
    // halves' two blocks per wave at 4 steps: still behind the one-board kernel at 256; at 8 they spill.)
    constexpr int PF = NB == 1 ? AZ_PART_PF : hk::PF;
    static_assert(NB * NP * NWV == 16 && SPX % SPI == 0 && SPX % PF == 0, "part kernel config");
    __shared__ __attribute__((aligned(16))) uint4 lds[LDS_U4];
    char* const l = reinterpret_cast<char*>(lds);
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // all parts of a board on one XCD (workgroups go round-robin over the 8 XCDs), one after the other
    const int bid = blockIdx.x;
    int board, part;
    if (B % 8 == 0) {
        const int j = bid >> 3;
        part = j % NP;
        board = (j / NP) * 8 + (bid & 7);
    } else {
        part = bid % NP;
        board = bid / NP;
    }
    board = vgpr_index(board);
    const size_t row0 = (size_t)board * 64;
    const int cb0 = (part * NWV + w) * NB;               // this wave's first 16-channel output block
    unsigned long long* const tr = trb && w == 0 ? trb + (size_t)blockIdx.x * 8 : nullptr;
    wino_stamp(tr, 0);
#ifdef AZ_TOWER_TRACE
    if (tr && lane == 0) {
        tr[4] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        tr[5] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));
    }
#endif
    float invR = 0.0f;
    if constexpr (XIN == 2) invR = 1.0f / (bb.nglob ? bb.nglob[vgpr_index(0)] : (float)bb.R);
    // zero rows; the staging's parameters
    for (int c = tid; c < PADU; c += 256)
#pragma unroll
        for (int s = 0; s < 3; s++) lds[s * (SLOT + PADU) + c] = make_uint4(0, 0, 0, 0);
    if constexpr (XIN != 0) {
        float4* par = reinterpret_cast<float4*>(l + SLOTS * 16);
        const float* src[5] = {XIN == 1 ? bn.mean : bb.mean, XIN == 1 ? bn.stdv : bb.stdv,
                               XIN == 1 ? bn.gamma : bb.gamma, XIN == 1 ? bn.beta : bb.dgamma, XIN == 1 ? nullptr : bb.dbeta};
#pragma unroll
        for (int p = 0; p < (XIN == 1 ? 4 : 5); p++)
            if (tid < F / 4) par[64 * p + tid] = reinterpret_cast<const float4*>(src[p])[tid];
    }
    __syncthreads();
    HalfStage<XIN> sg;
    sg.issue(X, bn, bb, row0, tid, 0);
    sg.finish(l, bn, bb, invR, tid, 0, 0, part == 0);
    sg.issue(X, bn, bb, row0, tid, 1);
    sg.finish(l, bn, bb, invR, tid, 1, 1, part == 1 % NP);
#if AZ_HALF_ISSUE == 1
    sg.issue(X, bn, bb, row0, tid, 2);
#endif
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)U, (short)0, (int)ubytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rN = __builtin_amdgcn_make_buffer_rsrc((void*)U, (short)0, 0, 0x00020000);
    const int voff = (cb0 * 64 + lane) * 16;           // wino_voff: fragment (block, lane)
    f32x4 wr[PF][NB];
#pragma unroll
    for (int i = 0; i < PF; i++)
#pragma unroll
        for (int n = 0; n < NB; n++)
            wr[i][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rW, voff + n * 1024, i * 16 * 1024, 0));
    __syncthreads();
    const HalfXf xf{l, w, lane};
    float* const bsd = XIN == 2 ? bb.bsum + (size_t)board * 2 * F : nullptr;
    {
        f32x2 d0[4][2];
        xf.load(0, d0);
        xf.store(0, d0);
        if (XIN == 2 && part == 0 && w == 0) half_bsum(l, 0, lane, bsd);
    }
    __syncthreads();
    wino_stamp(tr, 1);
    const int l16 = lane & 15, h = lane >> 4;
    const int vrd = h * 256 + ((l16 ^ (2 * h)) * 16);
    f32x4 acc[16][NB];
#pragma unroll
    for (int x = 0; x < 16; x++)
#pragma unroll
        for (int n = 0; n < NB; n++) {
            f32x2 z0, z1;
            asm volatile("v_mov_b64 %0, 0" : "=v"(z0));
            asm volatile("v_mov_b64 %0, 0" : "=v"(z1));
            acc[x][n] = f32x4{z0.x, z0.y, z1.x, z1.y};
        }
#pragma unroll 1
    for (int c = 0; c < NCH; c++) {
        const int vb = VB0 + (c & 1) * VBYTES + vrd;
        const bool more = c + 1 < NCH, stg = c + 2 < NCH;
        f32x2 dn[4][2];
        f32x4 bq[LA];
#pragma unroll
        for (int i = 0; i < LA; i++) bq[i] = *reinterpret_cast<const f32x4*>(l + vb + i * XST);
#pragma unroll
        for (int s0t = 0; s0t < SPX; s0t += SPI) {
            f32x4 Bf[SPI], a[SPI][NB];
#pragma unroll
            for (int u = 0; u < SPI; u++) {
                const int st = s0t + u;
                Bf[u] = bq[st % LA];
                if (st + LA < SPX) bq[st % LA] = *reinterpret_cast<const f32x4*>(l + vb + (st + LA) * XST);
#pragma unroll
                for (int n = 0; n < NB; n++) a[u][n] = wr[st % PF][n];
                const bool nxt = st + PF >= SPX && !more;
                const int tn = c * SPX + st + PF;
                const int to = nxt ? tn - NCH * SPX : tn;
#pragma unroll
                for (int n = 0; n < NB; n++)
                    wr[st % PF][n] = __builtin_bit_cast(
                        f32x4, __builtin_amdgcn_raw_buffer_load_b128(nxt ? rN : rW, voff + n * 1024, WINO_WSTEP(to) * 16 * 1024, 0));
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int u = 0; u < SPI; u++)
#pragma unroll
                    for (int n = 0; n < NB; n++)
                        acc[s0t + u][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][n][s4], Bf[u][s4], acc[s0t + u][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < SPI; u++) {
                const int st = s0t + u;
#if AZ_HALF_ISSUE == 0
                if (st == 0 && stg) sg.issue(X, bn, bb, row0, tid, c + 2);
#endif
                if (st == 0 && more) xf.load((c + 1) & 1, dn);
                if (st == TSPLIT && more) {
                    xf.store((c + 1) & 1, dn);
                    if (XIN == 2 && (c + 1) % NP == part && w == 0) half_bsum(l, (c + 1) & 1, lane, bsd + (c + 1) * CH);
                }
                if (st == SPX - 1 && stg) sg.finish(l, bn, bb, invR, tid, c + 2, c & 1, (c + 2) % NP == part);
#if AZ_HALF_ISSUE == 1
                // the next staging's loads in flight across the barrier and the next chunk
                if (st == SPX - 1 && c + 3 < NCH) sg.issue(X, bn, bb, row0, tid, c + 3);
#endif
            }
        }
        if (more) __syncthreads();
    }
    wino_stamp(tr, 2);
    // output transform (wino_core's), then conv_wino_train_kernel's epilogue for these channels
    const int co0 = cb0 * 16 + h * 4;
    f32x4 y[NB][4];
#pragma unroll
    for (int n = 0; n < NB; n++) {
        const f32x4 bb4 = bias ? *reinterpret_cast<const f32x4*>(bias + co0 + n * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 2; p++) {
            f32x2 m[16];
#pragma unroll
            for (int x = 0; x < 16; x++) m[x] = p ? f32x2{acc[x][n][2], acc[x][n][3]} : f32x2{acc[x][n][0], acc[x][n][1]};
            const f32x2 br = p ? f32x2{bb4[2], bb4[3]} : f32x2{bb4[0], bb4[1]};
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
    const int ty = l16 >> 2, tx = l16 & 3;
    f32x4 s0[NB], s1[NB];
#pragma unroll
    for (int n = 0; n < NB; n++) {
        s0[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        s1[n] = s0[n];
        f32x4 mu = s0[n], sd = s0[n];
        if constexpr (STATS == 2) {
            mu = *reinterpret_cast<const f32x4*>(bs.mean + co0 + n * 16);
            sd = *reinterpret_cast<const f32x4*>(bs.stdv + co0 + n * 16);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const size_t o = (row0 + (2 * ty + (q >> 1)) * 8 + 2 * tx + (q & 1)) * F + co0 + n * 16;
            f32x4 v = y[n][q];
            if constexpr (ADD) v += *reinterpret_cast<const f32x4*>(addend + o);
            *reinterpret_cast<f32x4*>(Y + o) = v;
            if constexpr (STATS == 1) {
                y[n][q] = v;
                s0[n] += v;
            } else if constexpr (STATS == 2) {
                const f32x4 ov = *reinterpret_cast<const f32x4*>(bs.O + o);
                const f32x4 yb = *reinterpret_cast<const f32x4*>(bs.Ybn + o);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const float dz = ov[r] > 0.0f ? v[r] : 0.0f;
                    s0[n][r] += dz;
                    s1[n][r] += dz * ((yb[r] - mu[r]) / sd[r]);
                }
            }
        }
    }
    if constexpr (STATS != 0) {
#pragma unroll
        for (int n = 0; n < NB; n++) {
            s0[n] = sum16(s0[n]);
            if constexpr (STATS == 1) {
                const f32x4 mb = s0[n] / 64.0f;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const f32x4 d = y[n][q] - mb;
                    s1[n] += d * d;
                }
            }
            s1[n] = sum16(s1[n]);
            if (l16 == 0) {
                float* pb = bs.part + (size_t)board * 2 * F + co0 + n * 16;
                *reinterpret_cast<f32x4*>(pb) = s0[n];
                *reinterpret_cast<f32x4*>(pb + F) = s1[n];
            }
        }
    }
    wino_stamp(tr, 3);
}

// Winograd weights U = G g G^T (f64, rounded once to f32: the same arithmetic as net.hip's
// winograd_f32) of one F x F 3x3 conv in the burn layout w[co][ci][3][3], into the layout
// wino_core streams ([ci/16][xi][co/16][lane][4]); flip = 1: the data-grad conv's kernel
// g'[o = ci][i = co][ky][kx] = w[co][ci][2 - ky][2 - kx].  One thread per (output, input) pair.
// All residual convs of the step in one launch (80 launches of ~7 us were 2 % of the step):
// blockIdx.y = 2 conv + flip; conv j's weights at w + j wstride, its U at U + (2 j + flip) ustride.
__global__ void __launch_bounds__(256) wino_weights_kernel(const float* __restrict__ w0, size_t wstride, int F,
                                                           float* __restrict__ U0, size_t ustride) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x, flip = blockIdx.y & 1;
    const float* __restrict__ w = w0 + (blockIdx.y >> 1) * wstride;
    float* __restrict__ U = U0 + (size_t)blockIdx.y * ustride;
    if (idx >= F * F / 4) return;
    // thread -> (output o, four inputs i0 .. i0 + 3): U's innermost dimension is i % 4, so each
    // point is one 16-byte store, and a wave's 64 lanes -- (o % 16, (i % 16) / 4) of one 16 x 16
    // (o, i) block -- write 1 KB contiguous per point.  (Round 5: one i per thread with four-byte
    // stores: 145 us for the step's 80 transforms; this form 134 us, bit-identical.)  The arithmetic
    // per element is unchanged (f64, rounded once).
    const int l = idx & 63, wv = idx >> 6, CF = F / 16;
    const int o = (wv % CF) * 16 + (l & 15), i0 = (wv / CF) * 16 + (l >> 4) * 4;
    float gf[4][9];   // [i - i0][ky 3 + kx] of U's conv
    if (!flip) {      // the four kernels are 36 consecutive floats, 16-byte aligned
        const float4* src = reinterpret_cast<const float4*>(w + ((size_t)o * F + i0) * 9);
#pragma unroll
        for (int q = 0; q < 9; q++) {
            const float4 t = src[q];
            gf[(4 * q) / 9][(4 * q) % 9] = t.x;
            gf[(4 * q + 1) / 9][(4 * q + 1) % 9] = t.y;
            gf[(4 * q + 2) / 9][(4 * q + 2) % 9] = t.z;
            gf[(4 * q + 3) / 9][(4 * q + 3) % 9] = t.w;
        }
    } else {          // the data grad's flipped, transposed kernel
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int t = 0; t < 9; t++) gf[j][t] = w[((size_t)(i0 + j) * F + o) * 9 + 8 - t];
    }
    const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
#pragma unroll
    for (int a = 0; a < 4; a++) {
        double gg[4][3];
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int c = 0; c < 3; c++)
                gg[j][c] = G[a][0] * (double)gf[j][c] + G[a][1] * (double)gf[j][3 + c] + G[a][2] * (double)gf[j][6 + c];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            float u[4];
#pragma unroll
            for (int j = 0; j < 4; j++) u[j] = (float)(gg[j][0] * G[b][0] + gg[j][1] * G[b][1] + gg[j][2] * G[b][2]);
            const int step = (i0 / 16) * 16 + a * 4 + b;
            *reinterpret_cast<float4*>(U + (((size_t)step * CF + o / 16) * 64 + l) * 4) = make_float4(u[0], u[1], u[2], u[3]);
        }
    }
}

__global__ void repack3x3_kernel(const float* __restrict__ w, int co_n, int ci_n, int kpad, float* __restrict__ wf,
                                 float* __restrict__ wd) {
    const size_t n = (size_t)9 * kpad * co_n;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int co = (int)(e % co_n), k = (int)((e / co_n) % kpad), t = (int)(e / ((size_t)co_n * kpad));
        const float v = k < ci_n ? w[((size_t)co * ci_n + k) * 9 + t] : 0.0f;
        wf[e] = v;
        if (wd && k < ci_n) wd[((size_t)(8 - t) * co_n + co) * ci_n + k] = v;
    }
}

// The split reduction and dW = G^T dU G in one pass: dU[xi][e] = sum over splits s (in order) of
// partial[s][xi][e], e = ci F + co, then dW[co][ci] = G^T dU G in f64, rounded once, into the
// gradient's burn layout g[co][ci][3][3] (bit-identical to the round-3 reduce_kernel + separate
// transform, 13.4 + 5.7 us per conv, without the dU round trip).  Workgroup = 64 lanes x 4
// consecutive e x 16 waves, wave = point: each thread's split loads are independent 16-byte loads
// (round 5: 13.9 us per conv against 15.5 with one e per lane, bit-identical; round 6: the splits'
// loads 2 / 4 / 16 at a time, 14.0 / 14.4 / 16.2 against 14.1 us -- bandwidth-, not latency-bound;
// a 4 ci x 64 co tile
// written as contiguous runs per co measured 23.4: too few workgroups), the points meet in LDS,
// waves 0-11 = (element of the four, kernel row ky).  (Round 5: a 256-thread form -- which would
// fit beside a Winograd conv workgroup on its CU -- on a second stream beside the next data-grad
// conv measured slower than in sequence, 22.72 vs 22.20 ms per step, as did the whole weight grad
// on a second stream (22.67 vs 22.62): its 256-VGPR workgroups hold their CUs for the whole GEMM,
// so the data-grad chain's small kernels queued behind them.  Not kept.)
__global__ void __launch_bounds__(1024) wino_wgrad_reduce_out_kernel(const float* __restrict__ partial, int splits,
                                                                      int F, float* __restrict__ g) {
    __shared__ float4 su[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t n4 = (size_t)F * F / 4, e4 = (size_t)blockIdx.x * 64 + lane;
    const float4* P4 = reinterpret_cast<const float4*>(partial);
    {
        const int xi = w;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = 0; k < splits; k++) {
            const float4 v = P4[((size_t)k * 16 + xi) * n4 + e4];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        su[xi][lane] = s;
    }
    __syncthreads();
    if (w >= 12) return;
    const int ky = w % 3, part = w / 3;   // wave: kernel row ky of element part of the lane's four
    const size_t e = e4 * 4 + part;
    const int co = (int)(e % F), ci = (int)(e / F);
    const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    auto u = [&](int x) { const float4 q = su[x][lane]; return (double)(part == 0 ? q.x : part == 1 ? q.y : part == 2 ? q.z : q.w); };
    double tg[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        tg[j] = G[0][ky] * u(j) + G[1][ky] * u(4 + j) + G[2][ky] * u(8 + j) + G[3][ky] * u(12 + j);
#pragma unroll
    for (int kx = 0; kx < 3; kx++)
        g[((size_t)co * F + ci) * 9 + ky * 3 + kx] =
            (float)(tg[0] * G[0][kx] + tg[1] * G[1][kx] + tg[2] * G[2][kx] + tg[3] * G[3][kx]);
}

// dWf[t][k][co] -> grad [co][ci][3][3]
__global__ void unpack3x3_kernel(const float* __restrict__ dwf, int co_n, int ci_n, int kpad, float* __restrict__ g) {
    const size_t n = (size_t)co_n * ci_n * 9;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int t = (int)(e % 9), ci = (int)((e / 9) % ci_n), co = (int)(e / ((size_t)9 * ci_n));
        g[e] = dwf[((size_t)t * kpad + ci) * co_n + co];
    }
}

// generic 2-D transpose with zero padding: dst[c][r] (ld_dst) = src[r][c] for r < rows, c < cols
__global__ void transpose_kernel(const float* __restrict__ src, int rows, int cols, float* __restrict__ dst, int ld_dst,
                                 int dst_rows) {
    const size_t n = (size_t)dst_rows * ld_dst;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(e / ld_dst), r = (int)(e % ld_dst);
        dst[e] = (c < cols && r < rows) ? src[(size_t)r * cols + c] : 0.0f;
    }
}

// ------------------------------------------------------------------ optimizer
// burn AdamW with GradientClipping::Value(1.0): g = clamp(grad*scale, -1, 1);
// m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g^2; update = (m/bc1) / (sqrt(v/bc2) + eps);
// p = p*(1 - lr*wd) - lr*update.  Running statistics (mask 0) are not parameters.
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, const uint8_t* __restrict__ mask, size_t n, float gscale,
                             float decay_mul, float lr, float bc1, float bc2) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        if (!mask[e]) continue;
        const float gr = fminf(fmaxf(g[e] * gscale, -1.0f), 1.0f);
        const float m1 = m[e] * 0.9f + gr * (1.0f - 0.9f);
        const float m2 = v[e] * 0.999f + (gr * gr) * (1.0f - 0.999f);
        m[e] = m1;
        v[e] = m2;
        const float upd = (m1 / bc1) / (sqrtf(m2 / bc2) + 1e-5f);
        p[e] = p[e] * decay_mul - upd * lr;
    }
}

// gather / scatter the running statistics (mask 2) into a contiguous buffer for the all-reduce
__global__ void stats_pack_kernel(float* __restrict__ p, const uint32_t* __restrict__ idx, int n, float* __restrict__ buf,
                                  int unpack, float scale) {
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        if (unpack) p[idx[e]] = buf[e] * scale;
        else buf[e] = p[idx[e]];
    }
}

}  // namespace tr

// ====================================================================== host side
namespace {

inline int grid_for(size_t n, int per = 256) {
    size_t g = (n + per - 1) / per;
    return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

struct Seg { size_t off, n; };

// flat parameter layout of include/az.h (az_net_num_params; azchess.agent.param_shapes)
struct Layout {
    struct Conv { size_t w, b, bn; int cin, cout, k; };
    std::vector<Conv> tower;          // input conv, then conv1/conv2 of every block
    size_t p1w, p1b, pbn, p2w, p2b, vw, vb, vbn, l1w, l1b, l2w, l2b, total;
    static Layout make(int B, int F) {
        Layout L;
        size_t o = 0;
        auto conv = [&](int cin, int cout, int k) {
            Conv c;
            c.cin = cin; c.cout = cout; c.k = k;
            c.w = o; o += (size_t)cout * cin * k * k;
            c.b = o; o += cout;
            c.bn = o; o += 4 * (size_t)cout;
            return c;
        };
        L.tower.push_back(conv(19, F, 3));
        for (int b = 0; b < 2 * B; b++) L.tower.push_back(conv(F, F, 3));
        L.p1w = o; o += 32 * (size_t)F; L.p1b = o; o += 32; L.pbn = o; o += 4 * 32;
        L.p2w = o; o += 64 * 32; L.p2b = o; o += 64;
        L.vw = o; o += 8 * (size_t)F; L.vb = o; o += 8; L.vbn = o; o += 4 * 8;
        L.l1w = o; o += 512 * 64; L.l1b = o; o += 64;
        L.l2w = o; o += 64; L.l2b = o; o += 1;
        L.total = o;
        return L;
    }
};

}  // namespace

struct Trainer {
    int blocks = 0, F = 0, Bmax = 0, device = 0;
    hipStream_t st = nullptr;
    Layout L;
    size_t np = 0;
    float *p = nullptr, *g = nullptr, *m = nullptr, *v = nullptr;
    uint8_t* mask = nullptr;
    long long t = 0;                         // AdamW time (burn AdaptiveMomentumWState::time)
    int last_batch = 0;
    // repacked weights
    std::vector<float*> wf, wd;
    // Winograd weights of the residual convs (F = 256): forward and data grad (env AZ_TRAIN_WINOGRAD=0: off)
    bool wino = false;
    std::vector<float*> uf, ud;              // conv i's forward / data-grad U: ubase + (2 (i - 1) + {0, 1}) ubytes
    float* ubase = nullptr;
    size_t ubytes = 0;
    float *w40f = nullptr, *w40d = nullptr, *b40 = nullptr, *wp2f = nullptr, *w1d = nullptr;
    // saved activations (R = B*64 rows)
    float* x0 = nullptr;                     // [R][X0C] input planes
    std::vector<float*> xs, y1, hh, y2;      // xs[0..blocks], y1/hh/y2[blocks]
    float *y0 = nullptr, *y40 = nullptr, *a40 = nullptr, *logits = nullptr, *vflat = nullptr, *h1 = nullptr;
    // gradients of activations
    float *dx = nullptr, *dxn = nullptr, *dres = nullptr, *dy = nullptr, *dh = nullptr;
    float *da40 = nullptr, *dy40 = nullptr, *dlog = nullptr, *dvflat = nullptr, *dh1 = nullptr;
    // per-BN statistics kept for backward: mean/std [nbn][F]
    float *bmean = nullptr, *bstd = nullptr, *dgb = nullptr;
    // reduction scratch
    float *wpart = nullptr, *cpart = nullptr, *dwtmp = nullptr;
    float* bpart = nullptr;                  // per-board BN partials [Bmax][2][F] (tr::BoardStats)
    float* bsum = nullptr;                   // conv bias-grad partials of bn_back4_kernel [grid][2][C]
    size_t bsum_cap = 0;
    size_t wpart_cap = 0, dwtmp_cap = 0;
    int slot = 0;                            // per-BN statistics stride (>= every BN's channels)
    float *tpol = nullptr, *tval = nullptr, *planes = nullptr, *loss = nullptr, *vpart = nullptr;
    float* hloss = nullptr;                  // pinned [Bmax][2]
    float* hlossx = nullptr;                 // pinned [4]: the losses summed in the gradient all-reduce
    // data parallel: RCCL communicator, or a host-side reducer (az_trainer_set_host_reducer)
    ncclComm_t comm = nullptr;
    az_allreduce_fn host_reduce = nullptr;
    void* host_ctx = nullptr;
    std::vector<float> host_buf;
    int rank = 0, world = 1;
    uint32_t* stat_idx = nullptr; float* stat_buf = nullptr; int nstat = 0;
    // sharded batch (az_trainer_set_sharded): BatchNorm statistics, the BN backward sums and the
    // loss normalisation over every rank's rows; xfwd [world][2 slot + 1] forward exchange,
    // xback [2 slot] backward exchange, nglob the global row count (device), lossx the losses
    bool sharded = false;
    float *xfwd = nullptr, *xback = nullptr, *xsum = nullptr, *nglob = nullptr, *lossx = nullptr;
    size_t xbs = 0;                          // floats per rank slot of xback
    int xfwd_world = 0;
    // az_trainer_step in sharded mode: the losses ride in the gradient all-reduce (g[np .. np + 3])
    bool loss_in_grad = false;
    float loss_out[2] = {0.0f, 0.0f};
    // every exchange (collective or host reduction) of the steps since the last read: count, and
    // HIP events around each one on the trainer stream (a pool of pairs, summed after each step)
    long long n_exchanges = 0, steps_exchanged = 0;
    double exchange_ms = 0.0;
    bool xtime = false;                      // events around each exchange (az_trainer_time_exchanges): they
                                             // cost ~3 us of queue time each, so timing is opt-in
    std::vector<hipEvent_t> xev;
    int xev_used = 0;
    bool fuse_bn = true;                     // BN apply / backward staged in the next Winograd conv (env AZ_TRAIN_FUSE_BN=0: off)
    bool orc = true;                         // O's sign recomputed where no residual (env AZ_TRAIN_ORC=0: off)
    int half = -1;                           // conv workgroups per board at small batches: -1 auto (4 when B <= 192),
                                             // 0 one per board, 2 / 4 always (env AZ_TRAIN_HALF)
    bool wgrad4 = true;                      // weight grad with one wave per SIMD (env AZ_TRAIN_WGRAD4=0: the 8-wave kernel)
    int wgrad_cosplit = 256;                 // batches up to this many boards split the one-wave weight grad's output
                                             // channels over two workgroups (env AZ_TRAIN_WGRAD_COSPLIT; round 6:
                                             // -4.5 / -3 / -0.8 % per step at 64 / 128 / 256, +0.7 % at 512)
    int wgrad_rows = 0;                      // A/B: a fixed weight-grad split size in rows (env AZ_TRAIN_WGRAD_ROWS)
    int wgrad_cosplit4 = 64;                 // ... and up to this many over four (env AZ_TRAIN_WGRAD_COSPLIT4; round 6: -0.9 %
                                             // at 64 against two, +1.5 % at 128)
    // the conv bias gradients of the tower's BatchNorms: bn_back4 partials per BN, summed in one
    // launch at the end of the backward (bias_dst[j] = gradient offset of BN j's conv bias)
    float* bsum_all = nullptr;
    size_t bsum_stride = 0;
    uint32_t* bias_dst = nullptr;
    std::vector<int> bias_pending;           // per BN: 0, or the partial blocks to sum
    std::vector<void*> allocs;
    // timing (HIP events on the trainer stream): whole steps and the gradient all-reduce
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    double step_ms = 0.0, allreduce_ms = 0.0;
    long long steps_timed = 0;

    float* alloc(size_t n) {
        void* q = nullptr;
        if (hipMalloc(&q, n * sizeof(float) + 16) != hipSuccess) return nullptr;
        allocs.push_back(q);
        return reinterpret_cast<float*>(q);
    }
    ~Trainer() {
        for (hipEvent_t e : ev) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : xev) if (e) (void)hipEventDestroy(e);
        if (comm) ncclCommDestroy(comm);
        for (void* q : allocs) (void)hipFree(q);
        if (hloss) (void)hipHostFree(hloss);
        if (hlossx) (void)hipHostFree(hlossx);
        if (st) (void)hipStreamDestroy(st);
    }
};

namespace {

constexpr int ROWS_PER_SPLIT = 512;   // weight-grad row split (8 boards)
#ifdef AZ_TOWER_TRACE
constexpr int TRACE_LAUNCHES = 128, TRACE_BOARDS = 4096;
unsigned long long* g_trace = nullptr;
int g_trace_n = 0;
#endif

int launch_conv(Trainer* T, int taps, const float* X, int ldx, int K, const float* W, int N, const float* bias,
                const float* addend, float* Y, int ldy, int R) {
    if (K % 16 || N % 16 || ldx % 4 || ldy % 4 || (taps == 9 && R % 64)) return fail("conv: bad shape");
    dim3 grid((R + tr::CM - 1) / tr::CM, (N + tr::CN - 1) / tr::CN);
    if (taps == 9) tr::conv_f32_kernel<9><<<grid, 256, 0, T->st>>>(X, ldx, K, W, N, bias, addend, Y, ldy, R);
    else tr::conv_f32_kernel<1><<<grid, 256, 0, T->st>>>(X, ldx, K, W, N, bias, addend, Y, ldy, R);
    return hipGetLastError() == hipSuccess ? 0 : fail("conv launch failed");
}

// the part kernel (NP workgroups per board) of launch_wino
template <int NPART>
int launch_wino_part(Trainer* T, const float* X, const uint4* U4, unsigned ub, const float* bias, const float* addend,
                     float* Y, int B, int stats, tr::BoardStats bs, tr::BnIn bn, tr::BnBack bb,
                     unsigned long long* htr) {   // phase stamps (trace build), one record per workgroup
    const unsigned g = (unsigned)(NPART * B);
    if (bn.out)
        tr::conv_wino_part_kernel<NPART, false, 1, 1><<<g, 256, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, htr);
    else if (bb.dy && addend)
        tr::conv_wino_part_kernel<NPART, true, 2, 2><<<g, 256, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, htr);
    else if (bb.dy)
        tr::conv_wino_part_kernel<NPART, false, 2, 2><<<g, 256, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, htr);
    else if (addend && stats == 2)
        tr::conv_wino_part_kernel<NPART, true, 2, 0><<<g, 256, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, htr);
    else if (addend && stats == 0)
        tr::conv_wino_part_kernel<NPART, true, 0, 0><<<g, 256, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, htr);
    else if (!addend && stats == 1)
        tr::conv_wino_part_kernel<NPART, false, 1, 0><<<g, 256, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, htr);
    else if (!addend && stats == 2)
        tr::conv_wino_part_kernel<NPART, false, 2, 0><<<g, 256, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, htr);
    else if (!addend && stats == 0)
        tr::conv_wino_part_kernel<NPART, false, 0, 0><<<g, 256, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, htr);
    else
        return fail("Winograd conv: unsupported statistics mode");
    return hipGetLastError() == hipSuccess ? 0 : fail("Winograd conv launch failed");
}

// Y = conv3x3(X, U) (+ bias) (+ addend) over B whole boards, Winograd (F = 256 residual convs);
// stats 1 / 2: per-board BN partials into bs.part (tr::BoardStats)
// bn.out non-null: X is the previous conv's pre-BN output, BatchNorm + ReLU (+ bn.res) applied in
// the staging and written to bn.out (tr::BnIn)
// bb.dy non-null: X is the BN backward's dout, the backward staged (tr::BnBack)
int launch_wino(Trainer* T, const float* X, const float* U, const float* bias, const float* addend, float* Y, int B,
                int stats = 0, tr::BoardStats bs = {}, tr::BnIn bn = {}, tr::BnBack bb = {}) {
    const uint4* U4 = reinterpret_cast<const uint4*>(U);
    const unsigned ub = (unsigned)T->ubytes;
    if (stats && !bs.part) return fail("Winograd conv: statistics without a buffer");
    if (bn.out && (addend || stats != 1)) return fail("Winograd conv: BatchNorm staging is a forward conv's");
    if (bb.dy && stats != 2) return fail("Winograd conv: the BN backward staging is a data-grad conv's");
    unsigned long long* trb = nullptr;   // phase stamps, trace build only (az_train_trace_read)
#ifdef AZ_TOWER_TRACE
    if (B <= TRACE_BOARDS) {
        if (!g_trace && hipMalloc(&g_trace, sizeof(unsigned long long) * TRACE_LAUNCHES * TRACE_BOARDS * 8) != hipSuccess)
            return fail("trace buffer");
        trb = g_trace + (size_t)(g_trace_n++ % TRACE_LAUNCHES) * TRACE_BOARDS * 8;
    }
#endif
    // small batches (the 512 / world shard of a sharded step): four quarter-channel workgroups per
    // board fill the CUs the one-board kernel leaves idle (conv_wino_part_kernel, bit-identical to
    // it).  Step at B = 64: 6.78 ms against 7.90 (halves) and 8.93 (one board); B = 128: 8.24 /
    // 8.93 / 9.87 (profiles/r06g_ab_parts_b*.txt); at B = 256 halves lose (12.37 vs 11.96, r06e).
    // With the quarters' deeper weight-ring prefetch (AZ_PART_PF): 7.49 / 8.66 / 9.58 at 128, and
    // 10.35 / 10.86 / 10.53 at 192, 12.90 / 12.06 / 11.60 at 256 (r06ad_ab_parts_b*.txt): quarters up
    // to 4B <= 3 x the CU count (B <= 192)
    const int np = T->half >= 0 ? T->half : (4 * B <= 3 * AZ_TRAIN_WG ? 4 : 0);
    // (trace build: one record per workgroup; trb holds TRACE_BOARDS >= 4 x 128)
    if (np == 2) return launch_wino_part<2>(T, X, U4, ub, bias, addend, Y, B, stats, bs, bn, bb, trb);
    if (np == 4) return launch_wino_part<4>(T, X, U4, ub, bias, addend, Y, B, stats, bs, bn, bb, trb);
    if (np != 0) return fail("Winograd conv: AZ_TRAIN_HALF must be -1, 0, 2 or 4");
    const unsigned wg = (unsigned)std::min(B, AZ_TRAIN_WG);   // persistent workgroups (one per CU)
    // ORC: O's sign recomputed (no residual: BN 0 and BN1s) where the host asks for it
    const int orc = (bb.dy && bb.beta ? 1 : 0) | (stats == 2 && bs.gamma ? 2 : 0);
    if (bn.out)
        tr::conv_wino_train_kernel<false, 1, 1><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, trb);
    else if (bb.dy && addend && orc == 1)   // conv1's data grad: BN1's backward, BN 2b's statistics
        tr::conv_wino_train_kernel<true, 2, 2, 1><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, trb);
    else if (bb.dy && addend && orc == 3)   // ... of block 0 (BN 0 has no residual either)
        tr::conv_wino_train_kernel<true, 2, 2, 3><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, trb);
    else if (bb.dy && !addend && orc == 2)  // conv2's data grad: BN2's backward, BN1's statistics
        tr::conv_wino_train_kernel<false, 2, 2, 2><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, trb);
    else if (bb.dy && addend)
        tr::conv_wino_train_kernel<true, 2, 2><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, trb);
    else if (bb.dy)
        tr::conv_wino_train_kernel<false, 2, 2><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, trb);
    else if (stats == 2 && bs.gamma && addend)   // unfused backward (AZ_TRAIN_FUSE_BN=0), conv1's data grad
        tr::conv_wino_train_kernel<true, 2, 0, 2><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, trb);
    else if (stats == 2 && bs.gamma)             // ... conv2's
        tr::conv_wino_train_kernel<false, 2, 0, 2><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, trb);
    else if (addend && stats == 2)
        tr::conv_wino_train_kernel<true, 2, 0><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, trb);
    else if (addend && stats == 0)
        tr::conv_wino_train_kernel<true, 0, 0><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, addend, Y, bs, bn, bb, B, trb);
    else if (!addend && stats == 1)
        tr::conv_wino_train_kernel<false, 1, 0><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, trb);
    else if (!addend && stats == 2)
        tr::conv_wino_train_kernel<false, 2, 0><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, trb);
    else if (!addend && stats == 0)
        tr::conv_wino_train_kernel<false, 0, 0><<<wg, 512, 0, T->st>>>(X, U4, ub, bias, nullptr, Y, bs, bn, bb, B, trb);
    else
        return fail("Winograd conv: unsupported statistics mode");
    return hipGetLastError() == hipSuccess ? 0 : fail("Winograd conv launch failed");
}

// dW[taps][K][N] = sum_r X[r+d_t][k] * DY[r][n]
int wgrad_rows_per_split(int taps, int R) { return taps == 9 || R >= 4096 ? ROWS_PER_SPLIT : 64; }
size_t wgrad_splits(int taps, int R) {
    const int rps = wgrad_rows_per_split(taps, R);
    return (size_t)((R + rps - 1) / rps);
}

// out_cap: elements the destination holds (taps*K*N must fit)
int launch_wgrad(Trainer* T, int taps, const float* X, int ldx, int K, const float* DY, int ldd, int N, int R,
                 float* out, size_t out_cap) {
    if (ldx % 4 || ldd % 4 || K % 4 || N % 16 || (taps == 9 && R % 64)) return fail("wgrad: bad shape");
    if ((size_t)taps * K * N > out_cap) return fail("wgrad: destination too small");
    if (wgrad_splits(taps, R) * taps * K * N > T->wpart_cap) return fail("wgrad: partial buffer too small");
    const int rps = wgrad_rows_per_split(taps, R);
    const int splits = (int)wgrad_splits(taps, R);
    dim3 grid((K + tr::GK - 1) / tr::GK, (N + tr::GN - 1) / tr::GN, splits);
    if (taps == 9 && K <= 32)   // the input conv (32 padded channels): half the k tile
        tr::wgrad_f32_kernel<9, 2><<<grid, 256, 0, T->st>>>(X, ldx, K, DY, ldd, N, R, rps, T->wpart, 1, 0, 0);
    else if (taps == 9) tr::wgrad_f32_kernel<9><<<grid, 256, 0, T->st>>>(X, ldx, K, DY, ldd, N, R, rps, T->wpart, 1, 0, 0);
    else tr::wgrad_f32_kernel<1><<<grid, 256, 0, T->st>>>(X, ldx, K, DY, ldd, N, R, rps, T->wpart, 1, 0, 0);
    const size_t n = (size_t)taps * K * N;
    tr::reduce_kernel<<<grid_for(n), 256, 0, T->st>>>(T->wpart, splits, n, out);
    return hipGetLastError() == hipSuccess ? 0 : fail("wgrad launch failed");
}

// Winograd weight grad of a residual F x F conv (input X, output gradient DY, B boards) into g
// F = 256 (wino_wgrad_gemm_kernel): the (board, tile) rows split into at most 16 splits of whole
// boards, 16 points each: 256 workgroups at B = 512 (512 rows per split), and still 256 at the
// 64 positions per rank of a world-8 sharded step (64 rows per split; round 6 -- a fixed 512-row
// split left 32 workgroups there, as slow as the whole 512 batch)
constexpr int WINO_GEMM_SPLITS = 16;
// nq output-channel parts per (split, point) (wino_wgrad_gemm4_kernel<2> at small batches): 16 / nq
// splits, so the workgroups stay 256 and the split partials shrink by nq.  fixed > 0 (A/B only, env
// AZ_TRAIN_WGRAD_ROWS): a fixed split size in rows (round 5: 512)
int wino_gemm_rows(int B, int nq, int fixed) {
    const int S = WINO_GEMM_SPLITS / nq;
    return fixed > 0 ? fixed : 16 * ((B + S - 1) / S);
}
size_t wino_gemm_splits(int B, int nq, int fixed) {
    const int rows = wino_gemm_rows(B, nq, fixed);
    return (size_t)((B * 16 + rows - 1) / rows);
}
size_t wino_gemm_splits_max(int Bmax, int fixed) {   // over B <= Bmax and nq
    return fixed > 0 ? wino_gemm_splits(Bmax, 1, fixed) : (size_t)std::min(Bmax, WINO_GEMM_SPLITS);
}
int launch_wino_wgrad(Trainer* T, const float* X, const float* DY, int B, float* g) {
    const int F = T->F, K = B * 16;
    if (F != 256) return fail("Winograd wgrad: F = 256 only");
    if (B > T->Bmax) return fail("Winograd wgrad: batch too large");
    const int nq = !T->wgrad4 ? 1 : B <= T->wgrad_cosplit4 ? 4 : B <= T->wgrad_cosplit ? 2 : 1;
    const int splits = (int)wino_gemm_splits(B, nq, T->wgrad_rows), rows = wino_gemm_rows(B, nq, T->wgrad_rows);
    if (splits * 16 * (size_t)F * F > T->wpart_cap) return fail("Winograd wgrad: partial buffer too small");
    if ((size_t)B * 64 * F * 4 >= (size_t)0x40000000) return fail("Winograd wgrad: batch too large for 32-bit offsets");
    if ((size_t)F * F % 256) return fail("Winograd wgrad: F * F must be a multiple of 256");
    const unsigned rblocks = (unsigned)((size_t)F * F / 256);
    if (nq == 4) tr::wino_wgrad_gemm4_kernel<4><<<dim3(splits, 16, 4), 256, 0, T->st>>>(X, DY, K, rows, T->wpart);
    else if (nq == 2) tr::wino_wgrad_gemm4_kernel<2><<<dim3(splits, 16, 2), 256, 0, T->st>>>(X, DY, K, rows, T->wpart);
    else if (T->wgrad4) tr::wino_wgrad_gemm4_kernel<1><<<dim3(splits, 16), 256, 0, T->st>>>(X, DY, K, rows, T->wpart);
    else tr::wino_wgrad_gemm_kernel<<<dim3(splits, 16), 512, 0, T->st>>>(X, DY, K, rows, T->wpart);
    tr::wino_wgrad_reduce_out_kernel<<<rblocks, 1024, 0, T->st>>>(T->wpart, splits, F, g);
    return hipGetLastError() == hipSuccess ? 0 : fail("Winograd wgrad launch failed");
}

int nblk_rows(int R) { return (R + tr::CS_ROWS - 1) / tr::CS_ROWS; }
#define TRY(x) do { if ((x) != 0) return -1; } while (0)

int host_allreduce(Trainer* T, float* d, size_t n, const char* what);
// sum of n floats at d over the ranks, on the trainer stream: RCCL, the host reducer, or nothing
// (one rank)
constexpr int XEV_PAIRS = 256;
// one exchange: counted, and bracketed by HIP events while az_trainer_time_exchanges is on
template <class Fn>
int exchange_run(Trainer* T, Fn&& fn) {
    if (!T->comm && !T->host_reduce) return 0;
    T->n_exchanges++;
    hipEvent_t* ev = nullptr;   // events around the exchange (none once the pool is used up)
    if (T->xtime && T->xev_used < XEV_PAIRS) {
        if (T->xev.empty()) {
            T->xev.assign(2 * XEV_PAIRS, nullptr);
            for (hipEvent_t& e : T->xev) AZ_HIP(hipEventCreate(&e));
        }
        ev = &T->xev[2 * T->xev_used++];
        AZ_HIP(hipEventRecord(ev[0], T->st));
    }
    if (fn() != 0) return -1;
    if (ev) AZ_HIP(hipEventRecord(ev[1], T->st));
    return 0;
}
int exchange(Trainer* T, float* d, size_t n, const char* what) {
    return exchange_run(T, [&]() -> int {
        if (T->comm) {
            if (ncclAllReduce(d, d, n, ncclFloat, ncclSum, T->comm, T->st) != ncclSuccess)
                return fail(std::string("ncclAllReduce (") + what + ") failed");
            return 0;
        }
        return host_allreduce(T, d, n, what);
    });
}
// every rank's slot of n floats, in rank order, into buf[world][n] (this rank's already at
// buf + rank n): an RCCL all-gather in place (one latency chain of world - 1 hops where an
// all-reduce takes two), or through the host reducer with the other slots zeroed (x + 0 = x
// exactly).  Round 6: the sharded BatchNorm exchanges are gathers; whatever is summed over ranks
// is then summed in rank order on the device (sum_slots_kernel), so RCCL and the host reducer
// compute the same floats, independent of RCCL's ring / tree order.
int gather_slots(Trainer* T, float* buf, size_t n, const char* what) {
    return exchange_run(T, [&]() -> int {
        if (T->comm) {
            if (ncclAllGather(buf + (size_t)T->rank * n, buf, n, ncclFloat, T->comm, T->st) != ncclSuccess)
                return fail(std::string("ncclAllGather (") + what + ") failed");
            return 0;
        }
        if (T->rank > 0) AZ_HIP(hipMemsetAsync(buf, 0, (size_t)T->rank * n * sizeof(float), T->st));
        if (T->rank + 1 < T->world)
            AZ_HIP(hipMemsetAsync(buf + (size_t)(T->rank + 1) * n, 0, (size_t)(T->world - 1 - T->rank) * n * sizeof(float),
                                  T->st));
        return host_allreduce(T, buf, (size_t)T->world * n, what);
    });
}
// after a step's final synchronisation: the exchanges' device time into exchange_ms
void exchange_times(Trainer* T) {
    for (int i = 0; i < T->xev_used; i++) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, T->xev[2 * i], T->xev[2 * i + 1]) == hipSuccess) T->exchange_ms += ms;
    }
    T->xev_used = 0;
}

// sharded batch: the exchange buffers for the current world (allocated on first use):
// xfwd [world][2 slot + 1] (forward statistics), xback [world][xbs] (backward sums, xbs = 2 slot:
// the tower's 2F or the heads' 80) + xsum [xbs] (their rank-order sums), nglob, lossx
int sharded_buffers(Trainer* T) {
    if (T->xfwd && T->xfwd_world == T->world) return 0;
    // every piece 256-byte aligned: the BN backward takes its four-channel path on the exchanged
    // sums exactly when it does on the rank's own (bn_vec), so one rank computes the plain step
    auto up = [](size_t k) { return (k + 63) & ~(size_t)63; };
    const size_t nf = up((size_t)T->world * (2 * T->slot + 1));
    T->xbs = up((size_t)2 * T->slot);
    const size_t nb = (size_t)T->world * T->xbs;
    float* q = T->alloc(nf + nb + T->xbs + 128);
    if (!q) return fail("sharded batch: out of device memory");
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, q) != hipSuccess || pa.device != T->device)
        return fail("sharded batch: exchange buffers not on the trainer's device");
    T->xfwd = q;
    T->xback = q + nf;
    T->xsum = T->xback + nb;
    T->nglob = T->xsum + T->xbs;
    T->lossx = T->nglob + 64;
    T->xfwd_world = T->world;
    return 0;
}

// the backward sums of n floats per rank: this rank's at xback + rank xbs (written by the caller),
// gathered, summed in rank order into xsum
int sum_over_ranks(Trainer* T, int n, const char* what) {
    TRY(gather_slots(T, T->xback, T->xbs, what));
    tr::sum_slots_kernel<<<(n + 255) / 256, 256, 0, T->st>>>(T->xback, T->world, T->xbs, n, T->xsum);
    return hipGetLastError() == hipSuccess ? 0 : fail("sum over ranks failed");
}

// the four-channel BN kernels apply: C a power of two in [4, 1024], ld and every pointer 16-byte
// aligned (the per-channel parameter vectors at channel 0 included: c is a multiple of 4)
bool bn_vec(int C, int ld, std::initializer_list<const float*> ptrs) {
    if (C < 4 || C > 1024 || (C & (C - 1)) || ld % 4) return false;
    for (const float* q : ptrs)
        if (((uintptr_t)q & 15) != 0) return false;
    return true;
}
// rows of 256 / (C / 4) per workgroup step; enough workgroups for 16 waves per CU at most
unsigned bn_grid(int C, int R) {
    const int rs = 256 / (C / 4);
    return (unsigned)std::max(1, std::min((R + rs - 1) / rs, 256 * 4));
}

// BN bi's normalisation + ReLU (+ residual) with the statistics in its slot: Y -> out
int bn_apply(Trainer* T, int bi, const float* Y, int ld, int C, int R, size_t bn_off, const float* res, float* out) {
    const float* P = T->p + bn_off;   // {gamma, beta, running_mean, running_var}
    const float* mean = T->bmean + (size_t)bi * T->slot;
    const float* sd = T->bstd + (size_t)bi * T->slot;
    if (bn_vec(C, ld, {Y, res, out, P, mean, sd}))
        tr::bn_apply4_kernel<<<bn_grid(C, R), 256, 0, T->st>>>(Y, ld, C, R, mean, sd, P, P + C, res, out);
    else
        tr::bn_apply_kernel<<<grid_for((size_t)R * C), 256, 0, T->st>>>(Y, ld, C, R, mean, sd, P, P + C, res, out);
    return hipGetLastError() == hipSuccess ? 0 : fail("bn forward failed");
}

// BatchNorm (training) + ReLU (+ residual): Y -> out; saves mean/std in slot `bi`
// bpart: per-board partials from the producing conv's epilogue (tr::BoardStats, STATS 1) instead
// of the two column-sum passes
// out == nullptr: the statistics only (the apply is staged in the next Winograd conv, tr::BnIn)
int bn_forward(Trainer* T, int bi, const float* Y, int ld, int C, int R, size_t bn_off, const float* res, float* out,
               const float* bpart = nullptr) {
    float* P = T->p + bn_off;   // {gamma, beta, running_mean, running_var}
    if (C > T->slot) return fail("bn: too many channels");
    float* mean = T->bmean + (size_t)bi * T->slot;
    float* sd = T->bstd + (size_t)bi * T->slot;
    if (T->sharded) {   // this rank's slot (sum, squared deviations from its mean, rows), exchange, combine
        const int ss = T->slot, rs = 2 * ss + 1;
        float* my = T->xfwd + (size_t)T->rank * rs;
        if (bpart) {
            if (R % 64 || ld != C) return fail("bn: board statistics need whole boards");
            tr::bn_local_kernel<<<tr::finalize_grid(C), tr::FIN_THREADS, 0, T->st>>>(bpart, R / 64, C, R, my, ss);
        } else {   // the column sums of the unsharded path: S, the rank's mean, M2 about it
            const int nb = nblk_rows(R);
            dim3 g(nb, (C + 63) / 64);
            tr::launch_colsum<0>(g, T->st, Y, ld, C, R, nullptr, nullptr, nullptr, nullptr, T->cpart,
                                 {tr::FIN_SUM, my, nullptr, nullptr, nullptr});
            tr::finalize_mean_kernel<<<tr::finalize_grid(C), tr::FIN_THREADS, 0, T->st>>>(T->cpart, nb, C, R, mean);
            tr::launch_colsum<1>(g, T->st, Y, ld, C, R, mean, nullptr, nullptr, nullptr, T->cpart,
                                 {tr::FIN_SUM, my + ss, nullptr, nullptr, nullptr});
            tr::set_value_kernel<<<1, 1, 0, T->st>>>(my + 2 * ss, (float)R);
        }
        TRY(gather_slots(T, T->xfwd, rs, "BatchNorm statistics"));
        tr::bn_global_kernel<<<(C + 255) / 256, 256, 0, T->st>>>(T->xfwd, T->world, C, ss, 0, mean, sd, P + 2 * C,
                                                                 P + 3 * C, bi == 0 ? T->nglob : nullptr);
    } else if (bpart) {
        if (R % 64 || ld != C) return fail("bn: board statistics need whole boards");
        tr::bn_board_var_kernel<<<tr::finalize_grid(C), tr::FIN_THREADS, 0, T->st>>>(bpart, R / 64, C, R, mean, sd, P + 2 * C,
                                                                        P + 3 * C);
    } else {
        const int nb = nblk_rows(R);
        dim3 g(nb, (C + 63) / 64);
        tr::launch_colsum<0>(g, T->st, Y, ld, C, R, nullptr, nullptr, nullptr, nullptr, T->cpart,
                             {tr::FIN_MEAN, mean, nullptr, nullptr, nullptr});
        tr::launch_colsum<1>(g, T->st, Y, ld, C, R, mean, nullptr, nullptr, nullptr, T->cpart,
                             {tr::FIN_VAR, sd, P + 2 * C, P + 3 * C, mean});
    }
    if (!out) return hipGetLastError() == hipSuccess ? 0 : fail("bn statistics failed");
    return bn_apply(T, bi, Y, ld, C, R, bn_off, res, out);
}

// sharded: the two head BatchNorms (policy: 32 channels at y40[:, 0:32], value: 8 at y40[:, 32:40],
// agent.rs:125,134) are independent, so they share ONE exchange -- their rank-local slots side by
// side, from one 40-channel column sum (a channel's sums do not depend on the width summed), one
// collective, then each combine (bn_global_kernel at its channel offset) and apply
int bn_forward_heads_sharded(Trainer* T, int bi, int R, size_t poff, size_t voff) {
    const int ss = T->slot, rs = 2 * ss + 1, C = 40;
    float* my = T->xfwd + (size_t)T->rank * rs;
    float* lmean = T->bmean + (size_t)bi * T->slot;   // scratch: this rank's 40 means (the combine overwrites it)
    const int nb = nblk_rows(R);
    dim3 g(nb, 1);
    tr::launch_colsum<0>(g, T->st, T->y40, 64, C, R, nullptr, nullptr, nullptr, nullptr, T->cpart,
                         {tr::FIN_SUM, my, nullptr, nullptr, nullptr});
    tr::finalize_mean_kernel<<<tr::finalize_grid(C), tr::FIN_THREADS, 0, T->st>>>(T->cpart, nb, C, R, lmean);
    tr::launch_colsum<1>(g, T->st, T->y40, 64, C, R, lmean, nullptr, nullptr, nullptr, T->cpart,
                         {tr::FIN_SUM, my + ss, nullptr, nullptr, nullptr});
    tr::set_value_kernel<<<1, 1, 0, T->st>>>(my + 2 * ss, (float)R);
    TRY(gather_slots(T, T->xfwd, rs, "head BatchNorm statistics"));
    float *Pp = T->p + poff, *Pv = T->p + voff;
    tr::bn_global_kernel<<<1, 256, 0, T->st>>>(T->xfwd, T->world, 32, ss, 0, T->bmean + (size_t)bi * ss,
                                               T->bstd + (size_t)bi * ss, Pp + 2 * 32, Pp + 3 * 32, nullptr);
    tr::bn_global_kernel<<<1, 256, 0, T->st>>>(T->xfwd, T->world, 8, ss, 32, T->bmean + (size_t)(bi + 1) * ss,
                                               T->bstd + (size_t)(bi + 1) * ss, Pv + 2 * 8, Pv + 3 * 8, nullptr);
    TRY(bn_apply(T, bi, T->y40, 64, 32, R, poff, nullptr, T->a40));
    return bn_apply(T, bi + 1, T->y40 + 32, 64, 8, R, voff, nullptr, T->a40 + 32);
}

// BatchNorm bi applied in the next Winograd conv's staging (statistics from bn_forward(out = null))
tr::BnIn bn_in(Trainer* T, int bi, size_t bn_off, const float* res, float* out) {
    const float* P = T->p + bn_off;
    return tr::BnIn{T->bmean + (size_t)bi * T->slot, T->bstd + (size_t)bi * T->slot, P, P + T->F, res, out};
}

// BN backward: dout (grad of the ReLU output O), pre-BN Y -> dy; dgamma/dbeta into the grad buffer
// bpart: per-board dz / dz*yhat sums from the conv that produced dout (tr::BoardStats, STATS 2)
// bias: the producing conv's bias gradient (sum of dy over rows), fused into the BN backward
int bias_grad(Trainer* T, const float* dy, int ld, int C, int R, float* dst);
// the BN backward's sums: dgamma / dbeta of this rank into the gradient (from the producing conv's
// per-board partials, or column sums), then -- sharded -- their global sums through xback;
// *ug / *ub: the sums the backward itself uses
int bn_back_sums(Trainer* T, int bi, const float* dout, const float* O, const float* Y, int ld, int C, int R,
                 size_t bn_off, const float* bpart, const float** ug_out, const float** ub_out, bool xchg = true) {
    const float* mean = T->bmean + (size_t)bi * T->slot;
    const float* sd = T->bstd + (size_t)bi * T->slot;
    float* dgam = T->g + bn_off;
    float* dbet = T->g + bn_off + C;
    float* my = T->sharded && xchg ? T->xback + (size_t)T->rank * T->xbs : nullptr;
    if (bpart) {
        if (R % 64 || ld != C) return fail("bn: board statistics need whole boards");
        tr::finalize_bnback_kernel<<<tr::finalize_grid(C), tr::FIN_THREADS, 0, T->st>>>(bpart, R / 64, C, dgam, dbet, my);
    } else {
        const int nb = nblk_rows(R);
        dim3 g(nb, (C + 63) / 64);
        tr::launch_colsum<2>(g, T->st, dout, ld, C, R, mean, sd, O, Y, T->cpart,
                             {tr::FIN_BNBACK, dgam, dbet, nullptr, nullptr});
    }
    // the gradient keeps this rank's dgamma / dbeta (summed over ranks with the rest of it);
    // sharded, the BN backward itself needs the global sums: exchanged through xback
    const float *ug = dgam, *ub = dbet;
    if (my) {
        if (!bpart) {   // the column-sum path finalized into the gradient only
            AZ_HIP(hipMemcpyAsync(my, dbet, C * sizeof(float), hipMemcpyDeviceToDevice, T->st));
            AZ_HIP(hipMemcpyAsync(my + C, dgam, C * sizeof(float), hipMemcpyDeviceToDevice, T->st));
        }
        TRY(sum_over_ranks(T, 2 * C, "BatchNorm backward sums"));
        ub = T->xsum;
        ug = T->xsum + C;
    }
    *ug_out = ug;
    *ub_out = ub;
    return hipGetLastError() == hipSuccess ? 0 : fail("bn backward sums failed");
}

// the BN backward of BN bi staged in the next Winograd data-grad conv (tr::BnBack): its sums here,
// the element-wise part in the conv's staging; bias partials per board, summed at the end
int bn_back_fused(Trainer* T, int bi, const float* dout, const float* O, const float* Y, int R, size_t bn_off,
                  const float* bpart, float* dy, float* dres, tr::BnBack* bb) {
    const int C = T->F, B = R / 64;
    const float *ug, *ub;
    TRY(bn_back_sums(T, bi, dout, O, Y, C, C, R, bn_off, bpart, &ug, &ub));
    if ((size_t)B * 2 * C > T->bsum_stride || bi >= (int)T->bias_pending.size()) return fail("bn: fused backward: bad shape");
    // BN 0 and the BN1s have no residual: the staging recomputes O's sign from Y (tr ORC bit 0)
    const bool orc = T->orc && (bi == 0 || bi % 2 == 1);
    *bb = tr::BnBack{O, Y, T->bmean + (size_t)bi * T->slot, T->bstd + (size_t)bi * T->slot, T->p + bn_off, ug, ub,
                     T->sharded ? T->nglob : nullptr, dy, dres, T->bsum_all + (size_t)bi * T->bsum_stride, R,
                     orc ? T->p + bn_off + C : nullptr};
    T->bias_pending[bi] = B;     // partials per board
    return 0;
}

int bn_back_apply(Trainer* T, int bi, const float* dout, const float* O, const float* Y, int ld, int C, int R,
                  size_t bn_off, float* dy, float* dres, float* bias, const float* ug, const float* ub);
int bn_backward(Trainer* T, int bi, const float* dout, const float* O, const float* Y, int ld, int C, int R,
                size_t bn_off, float* dy, float* dres, const float* bpart = nullptr, float* bias = nullptr) {
    const float *ug, *ub;
    TRY(bn_back_sums(T, bi, dout, O, Y, ld, C, R, bn_off, bpart, &ug, &ub));
    return bn_back_apply(T, bi, dout, O, Y, ld, C, R, bn_off, dy, dres, bias, ug, ub);
}

// sharded: the two head BatchNorms' backward sums share ONE exchange (xback = [dbeta_p 32 |
// dgamma_p 32 | dbeta_v 8 | dgamma_v 8], every piece 16-byte aligned as in bn_back_sums)
int bn_backward_heads_sharded(Trainer* T, int bi, int R, size_t poff, size_t voff) {
    const float *ug, *ub;
    TRY(bn_back_sums(T, bi, T->da40, T->a40, T->y40, 64, 32, R, poff, nullptr, &ug, &ub, false));
    TRY(bn_back_sums(T, bi + 1, T->da40 + 32, T->a40 + 32, T->y40 + 32, 64, 8, R, voff, nullptr, &ug, &ub, false));
    const size_t off[4] = {poff + 32, poff, voff + 8, voff};      // dbeta_p, dgamma_p, dbeta_v, dgamma_v
    const int pos[4] = {0, 32, 64, 72}, cnt[4] = {32, 32, 8, 8};
    float* my = T->xback + (size_t)T->rank * T->xbs;
    for (int k = 0; k < 4; k++)
        AZ_HIP(hipMemcpyAsync(my + pos[k], T->g + off[k], cnt[k] * sizeof(float), hipMemcpyDeviceToDevice, T->st));
    TRY(sum_over_ranks(T, 80, "head BatchNorm backward sums"));
    TRY(bn_back_apply(T, bi, T->da40, T->a40, T->y40, 64, 32, R, poff, T->dy40, nullptr, nullptr, T->xsum + 32,
                      T->xsum));
    return bn_back_apply(T, bi + 1, T->da40 + 32, T->a40 + 32, T->y40 + 32, 64, 8, R, voff, T->dy40 + 32, nullptr,
                         nullptr, T->xsum + 72, T->xsum + 64);
}

// the element-wise BN backward with the sums ug (dgamma) / ub (dbeta): dy (+ dres), bias partials
int bn_back_apply(Trainer* T, int bi, const float* dout, const float* O, const float* Y, int ld, int C, int R,
                  size_t bn_off, float* dy, float* dres, float* bias, const float* ug, const float* ub) {
    const float* mean = T->bmean + (size_t)bi * T->slot;
    const float* sd = T->bstd + (size_t)bi * T->slot;
    float* dgam = T->g + bn_off;
    float* dbet = T->g + bn_off + C;
    const float* nglob = T->sharded ? T->nglob : nullptr;
    if (bn_vec(C, ld, {dout, O, Y, dy, dres, T->p + bn_off, dgam, dbet, ug, ub, mean, sd})) {
        const unsigned g = bn_grid(C, R);
        if (bias && (size_t)g * 2 * C > T->bsum_cap) return fail("bn: bias partial buffer too small");
        // the tower's conv biases: partials kept per BN, summed at the end of the backward in one launch
        const bool batched = bias && T->bsum_all && bi < (int)T->bias_pending.size() && C == T->F;
        float* bs = batched ? T->bsum_all + (size_t)bi * T->bsum_stride : T->bsum;
        tr::bn_back4_kernel<<<g, 256, 0, T->st>>>(dout, O, Y, ld, C, R, mean, sd, T->p + bn_off, ug, ub, dy, dres,
                                                  bias ? bs : nullptr, nglob);
        if (batched) T->bias_pending[bi] = (int)g;
        else if (bias) tr::finalize_sum_kernel<<<tr::finalize_grid(C), tr::FIN_THREADS, 0, T->st>>>(T->bsum, (int)g, C, bias);
    } else {
        tr::bn_back_kernel<<<grid_for((size_t)R * C), 256, 0, T->st>>>(dout, O, Y, ld, C, R, mean, sd, T->p + bn_off,
                                                                       ug, ub, dy, dres, nglob);
        if (bias && bias_grad(T, dy, ld, C, R, bias) != 0) return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : fail("bn backward failed");
}

int bias_grad(Trainer* T, const float* dy, int ld, int C, int R, float* dst) {
    const int nb = nblk_rows(R);
    dim3 g(nb, (C + 63) / 64);
    tr::launch_colsum<0>(g, T->st, dy, ld, C, R, nullptr, nullptr, nullptr, nullptr, T->cpart,
                         {tr::FIN_SUM, dst, nullptr, nullptr, nullptr});
    return hipGetLastError() == hipSuccess ? 0 : fail("bias grad failed");
}

// defer_loss (az_trainer_step, sharded): the losses' exchange rides in the gradient all-reduce of
// the trainer_apply that follows (one dependent collective fewer); they are written there
int trainer_grads(Trainer* T, const float* planes, const float* tpol, const float* tval, int B, float* losses,
                  bool defer_loss = false) {
    if (B < 1 || B > T->Bmax) return fail("train: batch size out of range");
    T->last_batch = B;
    // the current device is per host thread (ranks as threads start on device 0): set it before
    // anything below allocates or launches
    AZ_HIP(hipSetDevice(T->device));
    if (T->sharded && sharded_buffers(T)) return -1;
    std::fill(T->bias_pending.begin(), T->bias_pending.end(), 0);
    AZ_HIP(hipEventRecord(T->ev[0], T->st));
    const int F = T->F, R = B * 64;
    hipStream_t st = T->st;
    const Layout& L = T->L;
    AZ_HIP(hipMemcpyAsync(T->planes, planes, (size_t)B * 19 * 64 * sizeof(float), hipMemcpyHostToDevice, st));
    AZ_HIP(hipMemcpyAsync(T->tpol, tpol, (size_t)B * 4096 * sizeof(float), hipMemcpyHostToDevice, st));
    AZ_HIP(hipMemcpyAsync(T->tval, tval, (size_t)B * sizeof(float), hipMemcpyHostToDevice, st));
    AZ_HIP(hipMemsetAsync(T->g, 0, T->np * sizeof(float), st));
    // weights of this step in GEMM layouts
    if (T->wino && T->blocks > 0) {  // residual convs: Winograd weights, forward and data grad, one launch
        const size_t wstride = L.tower.size() > 2 ? L.tower[2].w - L.tower[1].w : 0;
        if (F % 16) return fail("train: Winograd weights need F % 16 == 0");
        tr::wino_weights_kernel<<<dim3((unsigned)((F * F / 4 + 255) / 256), 2 * (L.tower.size() - 1)), 256, 0, st>>>(
            T->p + L.tower[1].w, wstride, F, T->ubase, T->ubytes / sizeof(float));
    }
    for (size_t i = 0; i < L.tower.size(); i++) {
        const auto& c = L.tower[i];
        if (i > 0 && T->wino) continue;
        const int kpad = i == 0 ? tr::X0C : F;
        tr::repack3x3_kernel<<<grid_for((size_t)9 * kpad * F), 256, 0, st>>>(T->p + c.w, F, c.cin, kpad, T->wf[i],
                                                                           i == 0 ? nullptr : T->wd[i]);
    }
    // heads 1x1 (policy_conv_1 | value_conv): w40d [64][F] = the two burn weights stacked
    // (rows >= 40 zero), w40f [F][64] its transpose
    AZ_HIP(hipMemsetAsync(T->w40d, 0, (size_t)64 * F * sizeof(float), st));
    AZ_HIP(hipMemcpyAsync(T->w40d, T->p + L.p1w, (size_t)32 * F * sizeof(float), hipMemcpyDeviceToDevice, st));
    AZ_HIP(hipMemcpyAsync(T->w40d + (size_t)32 * F, T->p + L.vw, (size_t)8 * F * sizeof(float), hipMemcpyDeviceToDevice, st));
    tr::transpose_kernel<<<grid_for((size_t)F * 64), 256, 0, st>>>(T->w40d, 64, F, T->w40f, 64, F);
    AZ_HIP(hipMemsetAsync(T->b40, 0, 64 * sizeof(float), st));
    AZ_HIP(hipMemcpyAsync(T->b40, T->p + L.p1b, 32 * sizeof(float), hipMemcpyDeviceToDevice, st));
    AZ_HIP(hipMemcpyAsync(T->b40 + 32, T->p + L.vb, 8 * sizeof(float), hipMemcpyDeviceToDevice, st));
    // policy_conv_2 [64][32] -> wp2f [32][64]; its data grad uses the burn layout as is
    tr::transpose_kernel<<<grid_for(32 * 64), 256, 0, st>>>(T->p + L.p2w, 64, 32, T->wp2f, 64, 32);
    // value_linear_1 [512][64] is already [K][N]; data grad needs [64][512]
    tr::transpose_kernel<<<grid_for(512 * 64), 256, 0, st>>>(T->p + L.l1w, 512, 64, T->w1d, 512, 64);

    // ---------------- forward (agent.rs:112-144, training-mode BatchNorm)
    tr::planes_kernel<<<grid_for((size_t)R * tr::X0C), 256, 0, st>>>(T->planes, B, T->x0);
    TRY(launch_conv(T, 9, T->x0, tr::X0C, tr::X0C, T->wf[0], F, T->p + L.tower[0].b, nullptr, T->y0, F, R));
    // Winograd tower: every BatchNorm but the last is applied in the next conv's staging (BnIn);
    // its statistics come from the producing conv's epilogue (bpart) except BN 0's
    const bool fuse = T->wino && T->fuse_bn && T->blocks > 0;
    TRY(bn_forward(T, 0, T->y0, F, F, R, L.tower[0].bn, nullptr, fuse ? nullptr : T->xs[0]));
    for (int b = 0; b < T->blocks; b++) {
        const auto& c1 = L.tower[1 + 2 * b];
        const auto& c2 = L.tower[2 + 2 * b];
        // Winograd convs hand their BN the per-board statistics (bpart) from their epilogue
        const float* bp = T->wino ? T->bpart : nullptr;
        if (fuse) {   // conv1's input: BN 0 (y0) or the previous block's BN2 (y2[b-1] + xs[b-1]) -> xs[b]
            const auto& pc = L.tower[2 * b];
            TRY(launch_wino(T, b == 0 ? T->y0 : T->y2[b - 1], T->uf[1 + 2 * b], T->p + c1.b, nullptr, T->y1[b], B, 1,
                            {T->bpart}, bn_in(T, 2 * b, pc.bn, b == 0 ? nullptr : T->xs[b - 1], T->xs[b])));
        } else if (T->wino) {
            TRY(launch_wino(T, T->xs[b], T->uf[1 + 2 * b], T->p + c1.b, nullptr, T->y1[b], B, 1, {T->bpart}));
        } else {
            TRY(launch_conv(T, 9, T->xs[b], F, F, T->wf[1 + 2 * b], F, T->p + c1.b, nullptr, T->y1[b], F, R));
        }
        TRY(bn_forward(T, 1 + 2 * b, T->y1[b], F, F, R, c1.bn, nullptr, fuse ? nullptr : T->hh[b], bp));
        if (fuse)     // conv2's input: BN1 of this block (y1[b]) -> hh[b]
            TRY(launch_wino(T, T->y1[b], T->uf[2 + 2 * b], T->p + c2.b, nullptr, T->y2[b], B, 1, {T->bpart},
                            bn_in(T, 1 + 2 * b, c1.bn, nullptr, T->hh[b])));
        else if (T->wino) TRY(launch_wino(T, T->hh[b], T->uf[2 + 2 * b], T->p + c2.b, nullptr, T->y2[b], B, 1, {T->bpart}));
        else TRY(launch_conv(T, 9, T->hh[b], F, F, T->wf[2 + 2 * b], F, T->p + c2.b, nullptr, T->y2[b], F, R));
        // the last block's BN2 feeds the heads' 1x1 convs: applied by its own pass
        const bool last = b == T->blocks - 1;
        TRY(bn_forward(T, 2 + 2 * b, T->y2[b], F, F, R, c2.bn, T->xs[b], (fuse && !last) ? nullptr : T->xs[b + 1], bp));
    }
    const float* body = T->xs[T->blocks];
    const int nbn = 1 + 2 * T->blocks;
    TRY(launch_conv(T, 1, body, F, F, T->w40f, 64, T->b40, nullptr, T->y40, 64, R));
    AZ_HIP(hipMemsetAsync(T->a40, 0, (size_t)R * 64 * sizeof(float), st));
    if (T->sharded) {
        TRY(bn_forward_heads_sharded(T, nbn, R, L.pbn, L.vbn));
    } else {
        TRY(bn_forward(T, nbn, T->y40, 64, 32, R, L.pbn, nullptr, T->a40));
        TRY(bn_forward(T, nbn + 1, T->y40 + 32, 64, 8, R, L.vbn, nullptr, T->a40 + 32));
    }
    TRY(launch_conv(T, 1, T->a40, 64, 32, T->wp2f, 64, T->p + L.p2b, nullptr, T->logits, 64, R));
    tr::vflat_kernel<<<grid_for((size_t)B * 512), 256, 0, st>>>(T->a40, T->vflat, B, 0);
    TRY(launch_conv(T, 1, T->vflat, 512, 512, T->p + L.l1w, 64, T->p + L.l1b, nullptr, T->h1, 64, B));
    // ---------------- loss + head tails
    tr::loss_kernel<<<B, 256, 0, st>>>(T->logits, T->tpol, T->h1, T->tval, T->p + L.l2w, T->p + L.l2b, B, T->dlog,
                                       T->dh1, T->loss, T->vpart, T->sharded ? T->nglob : nullptr);
    {   // value_linear_2 grads: sum over boards of the per-board partials
        const int nb = nblk_rows(B);
        dim3 g(nb, 2);
        tr::colsum_kernel<0><<<g, 256, 0, st>>>(T->vpart, 65, 65, B, nullptr, nullptr, nullptr, nullptr, T->cpart);
        tr::finalize_sum_kernel<<<tr::finalize_grid(65), tr::FIN_THREADS, 0, st>>>(T->cpart, nb, 65, T->dwtmp);
        AZ_HIP(hipMemcpyAsync(T->g + L.l2w, T->dwtmp, 64 * sizeof(float), hipMemcpyDeviceToDevice, st));
        AZ_HIP(hipMemcpyAsync(T->g + L.l2b, T->dwtmp + 64, sizeof(float), hipMemcpyDeviceToDevice, st));
    }
    // ---------------- backward
    // value_linear_1
    TRY(launch_wgrad(T, 1, T->vflat, 512, 512, T->dh1, 64, 64, B, T->g + L.l1w, 512 * 64));
    TRY(bias_grad(T, T->dh1, 64, 64, B, T->g + L.l1b));
    TRY(launch_conv(T, 1, T->dh1, 64, 64, T->w1d, 512, nullptr, nullptr, T->dvflat, 512, B));
    // policy_conv_2: dW[32][64] -> grad [64][32]
    TRY(launch_wgrad(T, 1, T->a40, 64, 32, T->dlog, 64, 64, R, T->dwtmp, T->dwtmp_cap));
    tr::transpose_kernel<<<grid_for(64 * 32), 256, 0, st>>>(T->dwtmp, 32, 64, T->g + L.p2w, 32, 64);
    TRY(bias_grad(T, T->dlog, 64, 64, R, T->g + L.p2b));
    AZ_HIP(hipMemsetAsync(T->da40, 0, (size_t)R * 64 * sizeof(float), st));
    TRY(launch_conv(T, 1, T->dlog, 64, 64, T->p + L.p2w, 32, nullptr, nullptr, T->da40, 64, R));
    tr::vflat_kernel<<<grid_for((size_t)B * 512), 256, 0, st>>>(T->da40, T->dvflat, B, 1);
    // head BatchNorms -> dy40 (cols >= 40 stay zero)
    AZ_HIP(hipMemsetAsync(T->dy40, 0, (size_t)R * 64 * sizeof(float), st));
    if (T->sharded) {
        TRY(bn_backward_heads_sharded(T, nbn, R, L.pbn, L.vbn));
    } else {
        TRY(bn_backward(T, nbn, T->da40, T->a40, T->y40, 64, 32, R, L.pbn, T->dy40, nullptr));
        TRY(bn_backward(T, nbn + 1, T->da40 + 32, T->a40 + 32, T->y40 + 32, 64, 8, R, L.vbn, T->dy40 + 32, nullptr));
    }
    // heads 1x1: dW[F][64] -> policy_conv_1 [32][F], value_conv [8][F]
    TRY(launch_wgrad(T, 1, body, F, F, T->dy40, 64, 64, R, T->dwtmp, (size_t)F * 64));
    tr::transpose_kernel<<<grid_for((size_t)40 * F), 256, 0, st>>>(T->dwtmp, F, 64, T->dwtmp + (size_t)F * 64, F, 40);
    AZ_HIP(hipMemcpyAsync(T->g + L.p1w, T->dwtmp + (size_t)F * 64, (size_t)32 * F * sizeof(float), hipMemcpyDeviceToDevice, st));
    AZ_HIP(hipMemcpyAsync(T->g + L.vw, T->dwtmp + (size_t)F * 64 + (size_t)32 * F, (size_t)8 * F * sizeof(float),
                          hipMemcpyDeviceToDevice, st));
    TRY(bias_grad(T, T->dy40, 64, 32, R, T->g + L.p1b));
    TRY(bias_grad(T, T->dy40 + 32, 64, 8, R, T->g + L.vb));
    TRY(launch_conv(T, 1, T->dy40, 64, 64, T->w40d, F, nullptr, nullptr, T->dx, F, R));
    // residual tower, last block first
    // dout of every BN but the last block's second comes from a Winograd data-grad conv, whose
    // epilogue leaves the BN backward's per-board sums in bpart (dx_stats: dx came with them)
    bool dx_stats = false;
    float* const dy = T->dy;   // each BN backward's dy: read by its conv's weight grad, then overwritten
    const bool fuseb = T->wino && T->fuse_bn;   // BN backward staged in the data-grad convs
    for (int b = T->blocks - 1; b >= 0; b--) {
        const auto& c1 = L.tower[1 + 2 * b];
        const auto& c2 = L.tower[2 + 2 * b];
        auto bstat = [&](int bi, const float* O, const float* Ybn) {
            // BN 0 and the BN1s have no residual: the epilogue recomputes O's sign (tr ORC bit 1)
            const bool orc = T->orc && (bi == 0 || bi % 2 == 1);
            const float* ga = orc ? T->p + L.tower[bi].bn : nullptr;
            return tr::BoardStats{T->bpart, O, Ybn, T->bmean + (size_t)bi * T->slot, T->bstd + (size_t)bi * T->slot, ga,
                                  orc ? ga + F : nullptr};
        };
        if (fuseb) {
            // BN2's backward (dout = dx) in conv2's data grad: dy (read by conv2's weight grad
            // after it), dz (-> dres), bias partials; conv2's output dh with BN1's sums in bpart
            tr::BnBack bb2;
            TRY(bn_back_fused(T, 2 + 2 * b, T->dx, T->xs[b + 1], T->y2[b], R, c2.bn, dx_stats ? T->bpart : nullptr, dy,
                              T->dres, &bb2));
            TRY(launch_wino(T, T->dx, T->ud[2 + 2 * b], nullptr, nullptr, T->dh, B, 2, bstat(1 + 2 * b, T->hh[b], T->y1[b]),
                            {}, bb2));
            TRY(launch_wino_wgrad(T, T->hh[b], dy, B, T->g + c2.w));
            // BN1's backward (dout = dh) in conv1's data grad (+ dres): dy, output dxn
            tr::BnBack bb1;
            TRY(bn_back_fused(T, 1 + 2 * b, T->dh, T->hh[b], T->y1[b], R, c1.bn, T->bpart, dy, nullptr, &bb1));
            TRY(launch_wino(T, T->dh, T->ud[1 + 2 * b], nullptr, T->dres, T->dxn, B, 2,
                            bstat(2 * b, T->xs[b], b > 0 ? T->y2[b - 1] : T->y0), {}, bb1));
            TRY(launch_wino_wgrad(T, T->xs[b], dy, B, T->g + c1.w));
            dx_stats = true;
            std::swap(T->dx, T->dxn);
            continue;
        }
        TRY(bn_backward(T, 2 + 2 * b, T->dx, T->xs[b + 1], T->y2[b], F, F, R, c2.bn, dy, T->dres,
                        dx_stats ? T->bpart : nullptr, T->g + c2.b));
        if (T->wino) {
            TRY(launch_wino_wgrad(T, T->hh[b], dy, B, T->g + c2.w));
        } else {
            TRY(launch_wgrad(T, 9, T->hh[b], F, F, dy, F, F, R, T->dwtmp, T->dwtmp_cap));
            tr::unpack3x3_kernel<<<grid_for((size_t)9 * F * F), 256, 0, st>>>(T->dwtmp, F, F, F, T->g + c2.w);
        }
        if (T->wino)
            TRY(launch_wino(T, dy, T->ud[2 + 2 * b], nullptr, nullptr, T->dh, B, 2, bstat(1 + 2 * b, T->hh[b], T->y1[b])));
        else TRY(launch_conv(T, 9, dy, F, F, T->wd[2 + 2 * b], F, nullptr, nullptr, T->dh, F, R));
        TRY(bn_backward(T, 1 + 2 * b, T->dh, T->hh[b], T->y1[b], F, F, R, c1.bn, dy, nullptr,
                        T->wino ? T->bpart : nullptr, T->g + c1.b));
        if (T->wino) {
            TRY(launch_wino_wgrad(T, T->xs[b], dy, B, T->g + c1.w));
        } else {
            TRY(launch_wgrad(T, 9, T->xs[b], F, F, dy, F, F, R, T->dwtmp, T->dwtmp_cap));
            tr::unpack3x3_kernel<<<grid_for((size_t)9 * F * F), 256, 0, st>>>(T->dwtmp, F, F, F, T->g + c1.w);
        }
        // dx is the gradient of block b's input: the output of BN 2b (BN 0 = the input conv's)
        if (T->wino)
            TRY(launch_wino(T, dy, T->ud[1 + 2 * b], nullptr, T->dres, T->dxn, B, 2, bstat(2 * b, T->xs[b],
                                                                                          b > 0 ? T->y2[b - 1] : T->y0)));
        else TRY(launch_conv(T, 9, dy, F, F, T->wd[1 + 2 * b], F, nullptr, T->dres, T->dxn, F, R));
        dx_stats = T->wino;
        std::swap(T->dx, T->dxn);
    }
    // input conv (no data grad)
    TRY(bn_backward(T, 0, T->dx, T->xs[0], T->y0, F, F, R, L.tower[0].bn, T->dy, nullptr, dx_stats ? T->bpart : nullptr,
                    T->g + L.tower[0].b));
    TRY(launch_wgrad(T, 9, T->x0, tr::X0C, tr::X0C, T->dy, F, F, R, T->dwtmp, T->dwtmp_cap));
    tr::unpack3x3_kernel<<<grid_for((size_t)9 * 19 * F), 256, 0, st>>>(T->dwtmp, F, 19, tr::X0C, T->g + L.tower[0].w);
    if (!T->bias_pending.empty()) {   // the tower's conv bias gradients: one launch for BNs 1..2B
        const int nt = (int)T->bias_pending.size();
        bool same = nt > 1;
        for (int j = 1; j < nt; j++) same = same && T->bias_pending[j] == T->bias_pending[1];
        const int j0 = same ? 1 : 0;
        if (same && T->bias_pending[1] > 0)
            tr::finalize_sum_batched_kernel<<<dim3(tr::finalize_grid(F), nt - 1), tr::FIN_THREADS, 0, st>>>(
                T->bsum_all + T->bsum_stride, T->bsum_stride, T->bias_pending[1], F, T->bias_dst + 1, T->g);
        for (int j = same ? 0 : j0; j < (same ? 1 : nt); j++)
            if (T->bias_pending[j] > 0)
                tr::finalize_sum_kernel<<<tr::finalize_grid(F), tr::FIN_THREADS, 0, st>>>(
                    T->bsum_all + (size_t)j * T->bsum_stride, T->bias_pending[j], F, T->g + L.tower[j].b);
        std::fill(T->bias_pending.begin(), T->bias_pending.end(), 0);
    }
    AZ_HIP(hipMemcpyAsync(T->hloss, T->loss, (size_t)B * 2 * sizeof(float), hipMemcpyDeviceToHost, st));
    AZ_HIP(hipStreamSynchronize(st));
    double pl = 0.0, vl = 0.0;
    for (int i = 0; i < B; i++) { pl += T->hloss[2 * i]; vl += T->hloss[2 * i + 1]; }
    double nb = B;
    T->loss_in_grad = false;
    if (T->sharded && (T->comm || T->host_reduce)) {   // means over the global batch
        float h[4] = {(float)pl, (float)vl, (float)B, 0.0f};
        if (defer_loss) {    // g[np .. np + 3], summed with the gradient (trainer_apply)
            AZ_HIP(hipMemcpyAsync(T->g + T->np, h, sizeof(h), hipMemcpyHostToDevice, st));
            AZ_HIP(hipStreamSynchronize(st));
            T->loss_in_grad = true;
            return 0;
        }
        AZ_HIP(hipMemcpyAsync(T->lossx, h, sizeof(h), hipMemcpyHostToDevice, st));
        AZ_HIP(hipStreamSynchronize(st));
        TRY(exchange(T, T->lossx, 4, "losses"));
        AZ_HIP(hipMemcpyAsync(h, T->lossx, sizeof(h), hipMemcpyDeviceToHost, st));
        AZ_HIP(hipStreamSynchronize(st));
        pl = h[0]; vl = h[1]; nb = h[2];
    }
    if (losses) {   // training.rs:281-282: means over the batch (policy, value)
        losses[0] = (float)(pl / nb);
        losses[1] = (float)(vl / nb);
    }
    return 0;
}

float powi_f32(float x, long long n) {   // Rust f32::powi (repeated squaring in f32)
    float r = 1.0f;
    while (n > 0) { if (n & 1) r *= x; x *= x; n >>= 1; }
    return r;
}

// the all-reduce (sum) of n floats at d through the caller's host reducer: device -> host, the
// reducer, host -> device, on the trainer stream
int host_allreduce(Trainer* T, float* d, size_t n, const char* what) {
    T->host_buf.resize(n);
    AZ_HIP(hipMemcpyAsync(T->host_buf.data(), d, n * sizeof(float), hipMemcpyDeviceToHost, T->st));
    AZ_HIP(hipStreamSynchronize(T->st));
    if (T->host_reduce(T->host_ctx, T->host_buf.data(), n) != 0)
        return fail(std::string("host reducer failed (") + what + ")");
    AZ_HIP(hipMemcpyAsync(d, T->host_buf.data(), n * sizeof(float), hipMemcpyHostToDevice, T->st));
    AZ_HIP(hipStreamSynchronize(T->st));
    return 0;
}

int trainer_apply(Trainer* T, double lr) {
    AZ_HIP(hipSetDevice(T->device));
    hipStream_t st = T->st;
    AZ_HIP(hipEventRecord(T->ev[1], st));
    // the gradient sum over ranks (a 1-rank communicator sums over itself: the identity, through
    // RCCL), with the deferred losses in its tail
    const bool lx = T->loss_in_grad;
    T->loss_in_grad = false;
    TRY(exchange(T, T->g, T->np + (lx ? 4 : 0), "gradients"));
    if (lx) AZ_HIP(hipMemcpyAsync(T->hlossx, T->g + T->np, 4 * sizeof(float), hipMemcpyDeviceToHost, st));
    AZ_HIP(hipEventRecord(T->ev[2], st));
    T->t++;
    const float bc1 = 1.0f - powi_f32(0.9f, T->t), bc2 = 1.0f - powi_f32(0.999f, T->t);
    const float decay_mul = (float)(1.0 - lr * 1e-4);   // WEIGHT_DECAY, parameters.rs:25
    // sharded: the summed gradient is already that of the global batch's mean loss (the loss and
    // the BN backward normalise by the global count); per-rank batches: the mean over ranks
    const float gscale = T->sharded ? 1.0f : 1.0f / (float)T->world;
    tr::adamw_kernel<<<grid_for(T->np), 256, 0, st>>>(T->p, T->g, T->m, T->v, T->mask, T->np, gscale, decay_mul,
                                                       (float)lr, bc1, bc2);
    // average the BatchNorm running statistics over ranks (sharded: every rank already holds the
    // same ones, updated from the global batch statistics)
    if ((T->comm || T->host_reduce) && !T->sharded) {
        tr::stats_pack_kernel<<<grid_for(T->nstat), 256, 0, st>>>(T->p, T->stat_idx, T->nstat, T->stat_buf, 0, 1.0f);
        TRY(exchange(T, T->stat_buf, (size_t)T->nstat, "running statistics"));
        tr::stats_pack_kernel<<<grid_for(T->nstat), 256, 0, st>>>(T->p, T->stat_idx, T->nstat, T->stat_buf, 1,
                                                                  1.0f / (float)T->world);
    }
    AZ_HIP(hipEventRecord(T->ev[3], st));
    AZ_HIP(hipGetLastError());
    AZ_HIP(hipStreamSynchronize(st));
    if (lx) {   // the global-batch means (as trainer_grads' separate exchange computes them)
        T->loss_out[0] = (float)((double)T->hlossx[0] / (double)T->hlossx[2]);
        T->loss_out[1] = (float)((double)T->hlossx[1] / (double)T->hlossx[2]);
    }
    float a = 0.0f, b = 0.0f;
    if (hipEventElapsedTime(&a, T->ev[0], T->ev[3]) == hipSuccess &&
        hipEventElapsedTime(&b, T->ev[1], T->ev[2]) == hipSuccess) {
        T->step_ms += a;
        T->allreduce_ms += b;
        T->steps_timed++;
    }
    exchange_times(T);
    if (T->comm || T->host_reduce) T->steps_exchanged++;
    return 0;
}

}  // namespace
}  // namespace azi

struct az_trainer { azi::Trainer* t; };

using namespace azi;

extern "C" {

double az_cyclical_lr(int iteration) {   // get_cyclical_lr, training.rs:424-441 (parameters.rs:20-24)
    const int decay_factor = iteration / 1000;
    const double mult = pow(10.0, -(double)decay_factor);
    const double base = 1e-3 * mult, mx = 1e-2 * mult;
    const int cur = iteration % 20;
    const double range = mx - base;
    if (cur <= 10) return base + (double)cur / 10.0 * range;
    return mx - (double)(cur - 10) / 10.0 * range;
}

int az_trainer_create(int blocks, int filters, const float* weights, size_t n, int max_batch, int device,
                      az_trainer** out) {
    if (!out || !weights || blocks < 0 || blocks > 40 || filters < 16 || filters % 16 || max_batch < 1)
        return fail("az_trainer_create: bad arguments (filters must be a multiple of 16)");
    if (n != az_net_num_params(blocks, filters)) return fail("az_trainer_create: weight count mismatch");
    AZ_HIP(hipSetDevice(device));
    Trainer* T = new Trainer();
    T->blocks = blocks; T->F = filters; T->Bmax = max_batch; T->device = device;
    T->L = Layout::make(blocks, filters);
    T->np = T->L.total;
    const int F = filters;
    const size_t R = (size_t)max_batch * 64;
    bool ok = hipStreamCreateWithFlags(&T->st, hipStreamNonBlocking) == hipSuccess;
    for (hipEvent_t& e : T->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    auto A = [&](size_t k) { float* q = T->alloc(k); ok = ok && q; return q; };
    T->p = A(T->np); T->g = A(T->np + 4); T->m = A(T->np); T->v = A(T->np);   // g: + the deferred losses
    void* mk = nullptr;
    ok = ok && hipMalloc(&mk, T->np) == hipSuccess;
    if (mk) T->allocs.push_back(mk);
    T->mask = reinterpret_cast<uint8_t*>(mk);
    const int nconv = 1 + 2 * blocks;
    T->wino = F == 256;
    if (const char* e = getenv("AZ_TRAIN_WINOGRAD")) T->wino = T->wino && atoi(e) != 0;
    // Winograd U per residual conv: 16 points x F x F + 8 zero ring steps of prefetch pad
    const size_t ufl = (size_t)16 * F * F + (size_t)8 * (F / 16) * 64 * 4;
    T->ubytes = ufl * sizeof(float);
    if (T->wino && nconv > 1) T->ubase = A(2 * (size_t)(nconv - 1) * ufl);
    for (int i = 0; i < nconv; i++) {
        const bool w9 = i == 0 || !T->wino;
        T->wf.push_back(w9 ? A((size_t)9 * (i == 0 ? tr::X0C : F) * F) : nullptr);
        T->wd.push_back(i == 0 || !w9 ? nullptr : A((size_t)9 * F * F));
        T->uf.push_back(i > 0 && T->ubase ? T->ubase + (size_t)(2 * (i - 1)) * ufl : nullptr);
        T->ud.push_back(i > 0 && T->ubase ? T->ubase + (size_t)(2 * (i - 1) + 1) * ufl : nullptr);
    }
    T->w40f = A((size_t)F * 64); T->w40d = A((size_t)64 * F); T->b40 = A(64); T->wp2f = A(32 * 64); T->w1d = A(64 * 512);
    T->x0 = A(R * tr::X0C);
    for (int b = 0; b <= blocks; b++) T->xs.push_back(A(R * F));
    for (int b = 0; b < blocks; b++) { T->y1.push_back(A(R * F)); T->hh.push_back(A(R * F)); T->y2.push_back(A(R * F)); }
    T->y0 = A(R * F); T->y40 = A(R * 64); T->a40 = A(R * 64); T->logits = A(R * 64);
    T->vflat = A((size_t)max_batch * 512); T->h1 = A((size_t)max_batch * 64);
    T->dx = A(R * F); T->dxn = A(R * F); T->dres = A(R * F); T->dy = A(R * F); T->dh = A(R * F);
    T->da40 = A(R * 64); T->dy40 = A(R * 64); T->dlog = A(R * 64);
    T->dvflat = A((size_t)max_batch * 512); T->dh1 = A((size_t)max_batch * 64);
    T->slot = std::max(F, 64);
    T->bmean = A((size_t)(nconv + 2) * T->slot); T->bstd = A((size_t)(nconv + 2) * T->slot);
    // weight-grad partials: the largest split count x output size over every wgrad launch
    // (split counts grow with the row count, so the maximum is at max_batch)
    const size_t s9 = wgrad_splits(9, (int)R), s1 = wgrad_splits(1, (int)R), sl = wgrad_splits(1, max_batch);
    size_t wp = s9 * 9 * 64 * (size_t)F;                                // input conv
    wp = std::max(wp, s9 * 9 * (size_t)F * F);                          // residual convs
    wp = std::max(wp, s1 * (size_t)F * 64);                             // heads 1x1
    wp = std::max(wp, s1 * 32 * 64);                                    // policy_conv_2
    wp = std::max(wp, sl * 512 * 64);                                   // value_linear_1
    if (const char* e = getenv("AZ_TRAIN_WGRAD_ROWS")) T->wgrad_rows = std::max(0, atoi(e) / 16 * 16);
    if (T->wino) {   // Winograd weight grads: [16][Bmax * 16][F] transforms, dU [16][F][F]
        wp = std::max(wp, wino_gemm_splits_max(max_batch, T->wgrad_rows) * 16 * (size_t)F * F);
    }
    T->wpart_cap = wp;
    T->wpart = A(wp);
    T->cpart = A((R / tr::CS_ROWS + 2) * 2 * (size_t)std::max(F, 65));
    T->bpart = A((size_t)max_batch * 2 * F);
    T->bsum_cap = (size_t)256 * 4 * 2 * std::max(F, 64);   // bn_grid's workgroup cap x [2][C]
    T->bsum = A(T->bsum_cap);
    if (T->wino) {   // per-BN bias partials of the tower (batched finalize) and the second dy
        // a slot holds either bn_back4's per-workgroup partials or the fused backward's per-board
        // ones (B x [2][F]): the larger of the two at max_batch
        T->bsum_stride = std::max(T->bsum_cap, (size_t)max_batch * 2 * F);
        T->bsum_all = A((size_t)nconv * T->bsum_stride);
        T->bias_pending.assign(nconv, 0);
    }
    // dW scratch: input conv [9][64][F], residual conv [9][F][F], heads [F][64] + its [40][F]
    // transpose, policy_conv_2 [32][64], value_linear_2 partial sums (65)
    T->dwtmp_cap = std::max({(size_t)9 * 64 * F, (size_t)9 * F * F, (size_t)F * 64 + 40 * (size_t)F, (size_t)32 * 64,
                             (size_t)65});
    T->dwtmp = A(T->dwtmp_cap);
    T->planes = A((size_t)max_batch * 19 * 64); T->tpol = A((size_t)max_batch * 4096); T->tval = A(max_batch);
    T->loss = A((size_t)max_batch * 2); T->vpart = A((size_t)max_batch * 65);
    ok = ok && hipHostMalloc((void**)&T->hloss, (size_t)max_batch * 2 * sizeof(float), 0) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&T->hlossx, 4 * sizeof(float), 0) == hipSuccess;
    if (const char* e = getenv("AZ_TRAIN_FUSE_BN")) T->fuse_bn = atoi(e) != 0;
    if (const char* e = getenv("AZ_TRAIN_ORC")) T->orc = atoi(e) != 0;
    if (const char* e = getenv("AZ_TRAIN_HALF")) T->half = atoi(e);
    if (const char* e = getenv("AZ_TRAIN_WGRAD4")) T->wgrad4 = atoi(e) != 0;
    if (const char* e = getenv("AZ_TRAIN_WGRAD_COSPLIT")) T->wgrad_cosplit = atoi(e);
    if (const char* e = getenv("AZ_TRAIN_WGRAD_COSPLIT4")) T->wgrad_cosplit4 = atoi(e);
    if (!ok) { delete T; return fail("az_trainer_create: out of device memory"); }
    // parameters, zero moments, trainable mask (BatchNorm running statistics are not parameters)
    std::vector<uint8_t> mask(T->np, 1);
    std::vector<uint32_t> sidx;
    auto bn_stats = [&](size_t off, int C) {
        for (int c = 0; c < 2 * C; c++) { mask[off + 2 * C + c] = 0; sidx.push_back((uint32_t)(off + 2 * C + c)); }
    };
    for (const auto& c : T->L.tower) bn_stats(c.bn, c.cout);
    bn_stats(T->L.pbn, 32);
    bn_stats(T->L.vbn, 8);
    T->nstat = (int)sidx.size();
    if (T->wino) {
        std::vector<uint32_t> bd;
        for (const auto& c : T->L.tower) bd.push_back((uint32_t)c.b);
        T->bias_dst = reinterpret_cast<uint32_t*>(T->alloc(bd.size()));
        if (!T->bias_dst || hipMemcpy(T->bias_dst, bd.data(), bd.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            delete T;
            return fail("az_trainer_create: out of device memory");
        }
    }
    T->stat_idx = reinterpret_cast<uint32_t*>(T->alloc(sidx.size()));
    T->stat_buf = T->alloc(sidx.size());
    if (!T->stat_idx || !T->stat_buf) { delete T; return fail("az_trainer_create: out of device memory"); }
    if (hipMemcpy(T->p, weights, T->np * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(T->mask, mask.data(), T->np, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(T->stat_idx, sidx.data(), sidx.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(T->m, 0, T->np * sizeof(float)) != hipSuccess || hipMemset(T->v, 0, T->np * sizeof(float)) != hipSuccess ||
        hipMemset(T->g, 0, T->np * sizeof(float)) != hipSuccess) {
        delete T;
        return fail("az_trainer_create: upload failed");
    }
    // the Winograd weight buffers' prefetch pad stays zero (the per-step transforms write the rest)
    if (T->ubase && hipMemset(T->ubase, 0, 2 * (size_t)(nconv - 1) * T->ubytes) != hipSuccess) {
        delete T;
        return fail("az_trainer_create: upload failed");
    }
    *out = new az_trainer{T};
    return 0;
}

int az_trainer_destroy(az_trainer* t) {
    if (!t) return 0;
    (void)hipSetDevice(t->t->device);
    delete t->t;
    delete t;
    return 0;
}

int az_trainer_compute_grads(az_trainer* t, const float* planes, const float* target_policy,
                             const float* target_value, int batch, float* losses) {
    if (!t || !planes || !target_policy || !target_value) return fail("null");
    return trainer_grads(t->t, planes, target_policy, target_value, batch, losses);
}

int az_trainer_apply(az_trainer* t, double lr) {
    if (!t) return fail("null");
    return trainer_apply(t->t, lr);
}

int az_trainer_step(az_trainer* t, const float* planes, const float* target_policy, const float* target_value,
                    int batch, double lr, float* losses) {
    if (!t || !planes || !target_policy || !target_value) return fail("null");
    if (trainer_grads(t->t, planes, target_policy, target_value, batch, losses, true) != 0) return -1;
    const bool lx = t->t->loss_in_grad;
    if (trainer_apply(t->t, lr) != 0) return -1;
    if (lx && losses) {
        losses[0] = t->t->loss_out[0];
        losses[1] = t->t->loss_out[1];
    }
    return 0;
}

int az_trainer_get_params(az_trainer* t, float* out, size_t n) {
    if (!t || !out || n != t->t->np) return fail("az_trainer_get_params: bad arguments");
    AZ_HIP(hipSetDevice(t->t->device));
    AZ_HIP(hipStreamSynchronize(t->t->st));
    AZ_HIP(hipMemcpy(out, t->t->p, n * sizeof(float), hipMemcpyDeviceToHost));
    return 0;
}

int az_trainer_get_grads(az_trainer* t, float* out, size_t n) {
    if (!t || !out || n != t->t->np) return fail("az_trainer_get_grads: bad arguments");
    AZ_HIP(hipSetDevice(t->t->device));
    AZ_HIP(hipStreamSynchronize(t->t->st));
    AZ_HIP(hipMemcpy(out, t->t->g, n * sizeof(float), hipMemcpyDeviceToHost));
    return 0;
}

int az_trainer_relu_output(az_trainer* t, int layer, float* out, size_t n) {
    if (!t || !out) return fail("null");
    Trainer* T = t->t;
    const size_t R = (size_t)T->last_batch * 64;
    const float* src = nullptr;
    size_t cnt = 0;
    const int nt = 1 + 2 * T->blocks;
    if (layer >= 0 && layer < nt) {           // x0, h0, x1, h1, ..., x_B (NHWC [R][F])
        src = layer == 0 ? T->xs[0] : (layer % 2 ? T->hh[(layer - 1) / 2] : T->xs[layer / 2]);
        cnt = R * T->F;
    } else if (layer == nt) {                  // heads: [R][64], columns 0..39 live
        src = T->a40; cnt = R * 64;
    } else if (layer == nt + 1) {              // value_linear_1 output before its ReLU [B][64]
        src = T->h1; cnt = (size_t)T->last_batch * 64;
    } else {
        return fail("az_trainer_relu_output: bad layer");
    }
    if (n != cnt) return fail("az_trainer_relu_output: size mismatch");
    AZ_HIP(hipSetDevice(T->device));
    AZ_HIP(hipStreamSynchronize(T->st));
    AZ_HIP(hipMemcpy(out, src, cnt * sizeof(float), hipMemcpyDeviceToHost));
    return 0;
}

int az_trainer_timing(az_trainer* t, double* step_ms, double* allreduce_ms, int64_t* steps, int reset) {
    if (!t) return fail("null");
    Trainer* T = t->t;
    if (step_ms) *step_ms = T->step_ms;
    if (allreduce_ms) *allreduce_ms = T->allreduce_ms;
    if (steps) *steps = T->steps_timed;
    if (reset) { T->step_ms = T->allreduce_ms = 0.0; T->steps_timed = 0; }
    return 0;
}

int az_comm_unique_id(void* out, int cap) {
    if (!out || cap < (int)sizeof(ncclUniqueId)) return fail("az_comm_unique_id: need 128 bytes");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return fail("ncclGetUniqueId failed");
    memcpy(out, &id, sizeof(id));
    return (int)sizeof(id);
}

int az_trainer_set_comm(az_trainer* t, const void* unique_id, int rank, int world) {
    if (!t || !unique_id || world < 1 || rank < 0 || rank >= world) return fail("az_trainer_set_comm: bad arguments");
    Trainer* T = t->t;
    AZ_HIP(hipSetDevice(T->device));
    if (T->comm) { ncclCommDestroy(T->comm); T->comm = nullptr; }
    T->host_reduce = nullptr;
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    if (ncclCommInitRank(&T->comm, world, id, rank) != ncclSuccess) return fail("ncclCommInitRank failed");
    T->rank = rank;
    T->world = world;
    return 0;
}

int az_trainer_set_sharded(az_trainer* t, int on) {
    if (!t) return fail("null");
    t->t->sharded = on != 0;
    return 0;
}

int az_trainer_time_exchanges(az_trainer* t, int on) {
    if (!t) return fail("null");
    t->t->xtime = on != 0;
    return 0;
}

int az_trainer_exchange_stats(az_trainer* t, int64_t* collectives, int64_t* steps, double* exchange_ms, int reset) {
    if (!t) return fail("null");
    Trainer* T = t->t;
    if (collectives) *collectives = T->n_exchanges;
    if (steps) *steps = T->steps_exchanged;
    if (exchange_ms) *exchange_ms = T->exchange_ms;
    if (reset) { T->n_exchanges = T->steps_exchanged = 0; T->exchange_ms = 0.0; }
    return 0;
}

int az_trainer_set_host_reducer(az_trainer* t, az_allreduce_fn fn, void* ctx, int rank, int world) {
    if (!t || !fn || world < 1 || rank < 0 || rank >= world) return fail("az_trainer_set_host_reducer: bad arguments");
    Trainer* T = t->t;
    AZ_HIP(hipSetDevice(T->device));
    if (T->comm) { ncclCommDestroy(T->comm); T->comm = nullptr; }
    T->host_reduce = fn;
    T->host_ctx = ctx;
    T->rank = rank;
    T->world = world;
    return 0;
}

}  // extern "C"

#ifdef AZ_TOWER_TRACE
// trace build only: the Winograd training convs' phase stamps, [launch % 128][board][8] (stamps 0-3:
// entry, staged, core done, exit; 4: HW_ID; 5: XCC_ID), and the number of launches so far
extern "C" int az_train_trace_read(unsigned long long* host, size_t n, int* launches) {
    if (launches) *launches = g_trace_n;
    if (!g_trace) return 0;
    const size_t all = (size_t)TRACE_LAUNCHES * TRACE_BOARDS * 8;
    AZ_HIP(hipDeviceSynchronize());
    AZ_HIP(hipMemcpy(host, g_trace, sizeof(unsigned long long) * (n < all ? n : all), hipMemcpyDeviceToHost));
    return 0;
}
#endif

// wgrad_dbg.hip -- debug harness for the fused-transform Winograd weight grad (wino_wgrad_gemm_kernel):
// the kernel, standalone, with its first stage's LDS image (xs = V rows, ds = M' rows) dumped
// after the staging barrier, against wino_wgrad_transform_kernel's Vt / Mt for the same board; then the
// whole partial against a host GEMM of Vt x Mt.  Splits "gather wrong" from "GEMM wrong" in one run.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/wgrad_dbg tools/wgrad_dbg.hip -lrccl
#include "../alphazero-chess_amd/csrc/train.hip"
#include <cstdio>
#include <vector>

namespace azi {
namespace tr {
// Winograd weight grad of a residual conv (F(2x2, 3x3), the forward conv's transforms
// transposed): with V = B^T d B the input patch transform (as in the forward) and
// M' = A dY A^T the 4x4 image of the tile's 2x2 output gradient (Y = A^T M A, so dL/dM = A dY A^T),
//   dU[xi][ci][co] = sum over (board, tile) of V[xi][ci] M'[xi][co]   (16 GEMMs, wgrad_f32_kernel)
//   dW[co][ci]     = G^T dU[co][ci] G                                   (U = G g G^T)
// 2.25x fewer MFMAs than the 9-tap implicit GEMM.  Vt[xi][k][ci], Mt[xi][k][co] with
// k = board * 16 + tile; one thread per (k, channel), channels fastest (coalesced).
// (The round-3 training step's transform pass; wino_wgrad_gemm_kernel now computes the same
// transforms in its staging, and this is the reference it is checked against.)
__global__ void __launch_bounds__(256) wino_wgrad_transform_kernel(const float* __restrict__ X,
                                                                   const float* __restrict__ DY, int F, int B,
                                                                   float* __restrict__ Vt, float* __restrict__ Mt) {
    const size_t K = (size_t)B * 16, n = K * F;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(e % F);
        const size_t k = e / F;
        const int t = (int)(k & 15), ty = t >> 2, tx = t & 3;
        const size_t b64 = (k >> 4) * 64;
        float d[4][4];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int r = 2 * ty - 1 + i, f = 2 * tx - 1 + j;
                d[i][j] = ((unsigned)r < 8u && (unsigned)f < 8u) ? X[(b64 + r * 8 + f) * F + c] : 0.0f;
            }
        float y[2][2];
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int bb = 0; bb < 2; bb++) y[a][bb] = DY[(b64 + (2 * ty + a) * 8 + 2 * tx + bb) * F + c];
        float tt[4][4], p[4][2];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            tt[0][j] = d[0][j] - d[2][j];
            tt[1][j] = d[1][j] + d[2][j];
            tt[2][j] = d[2][j] - d[1][j];
            tt[3][j] = d[1][j] - d[3][j];
        }
#pragma unroll
        for (int bb = 0; bb < 2; bb++) {
            p[0][bb] = y[0][bb];
            p[1][bb] = y[0][bb] + y[1][bb];
            p[2][bb] = y[0][bb] - y[1][bb];
            p[3][bb] = -y[1][bb];
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const float v[4] = {tt[r][0] - tt[r][2], tt[r][1] + tt[r][2], tt[r][2] - tt[r][1], tt[r][1] - tt[r][3]};
            const float m[4] = {p[r][0], p[r][0] + p[r][1], p[r][0] - p[r][1], -p[r][1]};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                Vt[((size_t)(r * 4 + q) * K + k) * F + c] = v[q];
                Mt[((size_t)(r * 4 + q) * K + k) * F + c] = m[q];
            }
        }
    }
}
}  // namespace tr
}  // namespace azi

// the library entry points train.hip refers to (not exercised here)
namespace azi { int fail(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); return -1; } }
extern "C" size_t az_net_num_params(int, int) { return 0; }

namespace dbg {
using azi::tr::f32x4;
constexpr int WG_S = 256 + 16;
__device__ __forceinline__ f32x4 wino_comb(int k, f32x4 a, f32x4 b) { return k == 1 ? a + b : k == 2 ? b - a : a - b; }

template <int VARIANT>
__global__ void __launch_bounds__(512)
fused_kernel(const float* __restrict__ X, const float* __restrict__ DY, int K, int rows_per_split,
             float* __restrict__ partial, float* __restrict__ dump) {
    constexpr int F = 256;
    __shared__ __attribute__((aligned(16))) float xs[16 * WG_S];
    __shared__ __attribute__((aligned(16))) float ds[16 * WG_S];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int split = blockIdx.x, xi = blockIdx.y, r = xi >> 2, q = xi & 3;
    const int i1 = r == 0 ? 0 : 1, i2 = r == 3 ? 3 : 2, j1 = q == 0 ? 0 : 1, j2 = q == 3 ? 3 : 2;
    const int rbeg = split * rows_per_split, rend = min(K, rbeg + rows_per_split);
    f32x4 acc[16][2];
#pragma unroll
    for (int b = 0; b < 16; b++)
#pragma unroll
        for (int n = 0; n < 2; n++) acc[b][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int c4 = (tid & 63) * 4, tp = tid >> 6;
    f32x4 xd[2][2][2], yv[2][2][2];
    auto fetch = [&](int rc) {
        const size_t b64 = (size_t)(rc >> 4) * 64;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int t = 2 * tp + u, ty = t >> 2, tx = t & 3;
#pragma unroll
            for (int ii = 0; ii < 2; ii++)
#pragma unroll
                for (int jj = 0; jj < 2; jj++) {
                    const int row = 2 * ty - 1 + (ii ? i2 : i1), col = 2 * tx - 1 + (jj ? j2 : j1);
                    xd[u][ii][jj] = ((unsigned)row < 8u && (unsigned)col < 8u)
                                        ? *reinterpret_cast<const f32x4*>(X + (b64 + row * 8 + col) * F + c4)
                                        : f32x4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int bb = 0; bb < 2; bb++)
                    yv[u][a][bb] = *reinterpret_cast<const f32x4*>(DY + (b64 + (2 * ty + a) * 8 + 2 * tx + bb) * F + c4);
        }
    };
    if (rbeg < rend) fetch(rbeg);
    for (int rc = rbeg; rc < rend; rc += 16) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int t = 2 * tp + u;
            const f32x4 tt1 = wino_comb(r, xd[u][0][0], xd[u][1][0]), tt2 = wino_comb(r, xd[u][0][1], xd[u][1][1]);
            const f32x4 v = wino_comb(q, tt1, tt2);
            f32x4 p[2];
            if constexpr (VARIANT == 0) {   // the select chain the patch used (miscompiled: r = 3 gives y0)
#pragma unroll
                for (int bb = 0; bb < 2; bb++) {
                    const f32x4 y0 = yv[u][0][bb], y1 = yv[u][1][bb];
                    p[bb] = r == 0 ? y0 : r == 1 ? y0 + y1 : r == 2 ? y0 - y1 : -y1;
                }
            } else {                        // coefficient form (train.hip)
                const float ra = r == 3 ? 0.0f : 1.0f, rb = r == 0 ? 0.0f : (r == 1 ? 1.0f : -1.0f);
#pragma unroll
                for (int bb = 0; bb < 2; bb++) p[bb] = yv[u][0][bb] * ra + yv[u][1][bb] * rb;
            }
            const float qa = q == 3 ? 0.0f : 1.0f, qb = q == 0 ? 0.0f : (q == 1 ? 1.0f : -1.0f);
            const f32x4 m = VARIANT == 0 ? (q == 0 ? p[0] : q == 1 ? p[0] + p[1] : q == 2 ? p[0] - p[1] : -p[1])
                                         : p[0] * qa + p[1] * qb;
            *reinterpret_cast<f32x4*>(xs + t * WG_S + c4) = v;
            *reinterpret_cast<f32x4*>(ds + t * WG_S + c4) = m;
        }
        __syncthreads();
        if (rc == rbeg && split == 0) {                    // the first stage's LDS image, as staged
            for (int e = tid; e < 16 * 256; e += 512) {
                dump[((size_t)xi * 2 + 0) * 16 * 256 + e] = xs[(e >> 8) * WG_S + (e & 255)];
                dump[((size_t)xi * 2 + 1) * 16 * 256 + e] = ds[(e >> 8) * WG_S + (e & 255)];
            }
        }
        if (rc + 16 < rend) fetch(rc + 16);
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            const int rq = qq * 4 + (lane >> 4);
            const float b0 = ds[rq * WG_S + 32 * w + (lane & 15)];
            const float b1 = ds[rq * WG_S + 32 * w + 16 + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(xs + rq * WG_S + 64 * j + 4 * (lane & 15));
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    acc[4 * j + c][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], b0, acc[4 * j + c][0], 0, 0, 0);
                    acc[4 * j + c][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], b1, acc[4 * j + c][1], 0, 0, 0);
                }
            }
        }
    }
    float* out = partial + ((size_t)split * 16 + xi) * F * F;
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int ci = 64 * j + 4 * (4 * (lane >> 4) + g) + c, co = 32 * w + 16 * n + (lane & 15);
                    out[(size_t)ci * F + co] = acc[4 * j + c][n][g];
                }
}
}  // namespace dbg

int main() {
    const int B = 2, F = 256, K = B * 16;
    std::vector<float> hx((size_t)B * 64 * F), hd((size_t)B * 64 * F);
    unsigned s = 1;
    for (auto& v : hx) { s = s * 1664525u + 1013904223u; v = (float)((s >> 8) & 0xffff) / 65536.f - 0.5f; }
    for (auto& v : hd) { s = s * 1664525u + 1013904223u; v = (float)((s >> 8) & 0xffff) / 65536.f - 0.5f; }
    float *x, *d, *vt, *mt, *part, *part2, *dump;
    hipMalloc(&x, hx.size() * 4); hipMalloc(&d, hd.size() * 4);
    hipMalloc(&vt, (size_t)16 * K * F * 4); hipMalloc(&mt, (size_t)16 * K * F * 4);
    hipMalloc(&part, (size_t)16 * F * F * 4); hipMalloc(&part2, (size_t)16 * F * F * 4);
    hipMalloc(&dump, (size_t)16 * 2 * 16 * 256 * 4);
    hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d, hd.data(), hd.size() * 4, hipMemcpyHostToDevice);
    azi::tr::wino_wgrad_transform_kernel<<<64, 256>>>(x, d, F, B, vt, mt);
    azi::tr::wino_wgrad_gemm_kernel<<<dim3(1, 16), 512>>>(x, d, K, 512, part2);    // the product kernel
    const int variant = getenv("WGDBG_VARIANT") ? atoi(getenv("WGDBG_VARIANT")) : 0;
    if (variant) dbg::fused_kernel<1><<<dim3(1, 16), 512>>>(x, d, K, 512, part, dump);
    else dbg::fused_kernel<0><<<dim3(1, 16), 512>>>(x, d, K, 512, part, dump);
    printf("variant %d (%s)\n", variant, variant ? "coefficients" : "select chain");
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
    std::vector<float> hv((size_t)16 * K * F), hm((size_t)16 * K * F), hp((size_t)16 * F * F), hp2(hp.size()),
        hdump((size_t)16 * 2 * 16 * 256);
    hipMemcpy(hv.data(), vt, hv.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hm.data(), mt, hm.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hp.data(), part, hp.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hp2.data(), part2, hp2.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hdump.data(), dump, hdump.size() * 4, hipMemcpyDeviceToHost);
    // (1) staging: the fused kernel's LDS rows of board 0 vs the transform kernel's Vt / Mt rows 0..15
    int bad_v = 0, bad_m = 0, shown = 0;
    for (int xi = 0; xi < 16; xi++)
        for (int t = 0; t < 16; t++)
            for (int c = 0; c < 256; c++) {
                const float gv = hdump[((size_t)xi * 2 + 0) * 4096 + t * 256 + c], rv = hv[((size_t)xi * K + t) * F + c];
                const float gm = hdump[((size_t)xi * 2 + 1) * 4096 + t * 256 + c], rm = hm[((size_t)xi * K + t) * F + c];
                if (gv != rv) { bad_v++; if (shown < 6) { printf("V xi %d tile %d c %d: lds %g transform %g\n", xi, t, c, gv, rv); shown++; } }
                if (gm != rm) { bad_m++; if (shown < 12) { printf("M xi %d tile %d c %d: lds %g transform %g\n", xi, t, c, gm, rm); shown++; } }
            }
    printf("staging: %d V and %d M' entries differ (of %d each)\n", bad_v, bad_m, 16 * 16 * 256);
    // (2) the GEMMs: this harness's kernel and the product kernel against the host GEMM of Vt x Mt
    double e1 = 0, e2 = 0, mr = 0;
    for (int xi = 0; xi < 16; xi++)
        for (int ci = 0; ci < F; ci++)
            for (int co = 0; co < F; co++) {
                double rr = 0;
                for (int k = 0; k < K; k++) rr += (double)hv[((size_t)xi * K + k) * F + ci] * hm[((size_t)xi * K + k) * F + co];
                const size_t o = ((size_t)xi * F + ci) * F + co;
                e1 = std::max(e1, fabs(hp[o] - rr));
                e2 = std::max(e2, fabs(hp2[o] - rr));
                mr = std::max(mr, fabs(rr));
            }
    printf("GEMM max error: harness %g, product %g (max |ref| %g)\n", e1, e2, mr);
    return (bad_v || bad_m || e1 > 1e-3 || e2 > 1e-3) ? 1 : 0;
}

// select_chain_repro.hip -- VERDICT r4 item 6: is the vector select chain that gave a wrong M'
// in the round-3/4 fused Winograd weight grad miscompiled for gfx950, or was the kernel at fault?
//
//   p = r == 0 ? y0 : r == 1 ? y0 + y1 : r == 2 ? y0 - y1 : -y1        (f32x4, r wave-uniform)
//
// Four kernels, each on the shapes of the original (tools/wgrad_dbg.hip VARIANT 0):
//   k_chain_uniform  r = blockIdx.y >> 2 (wave-uniform, an SGPR: the original's r = xi >> 2)
//   k_chain_lane     r = a per-lane value loaded from memory (a VGPR)
//   k_chain_staged   the original's full staging step: the chain for the row and the column
//                    combination (q), results written through LDS as the GEMM staged them
//   k_chain_loop     the staged form inside the software-pipelined board loop
// Result on MI355X / ROCm 7.2 (profiles/r05_select_chain.txt): all four are CORRECT -- the chain
// is not miscompiled in isolation.  The original kernel (tools/wgrad_dbg.hip, fused_kernel<0>:
// the same chain among the weight grad's MFMAs, 16 f32x4 loads in flight, 232+ VGPRs) still
// returns y0 for r = 3 on the GPU, and its ISA shows why: the structurized flow of the 4-way
// select computes the `-y1` arm only on the r < 2 path (where the r == 1 arm then overwrites
// it), so r == 3 falls through with the default y0 -- a code-generation fault that depends on
// the surrounding kernel (ISA excerpt: profiles/r05_select_chain_isa.txt).
// The host computes every element on the CPU and counts mismatches per r.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/select_chain_repro.hip
//        -o tools/select_chain_repro  (ISA: add --save-temps, or llvm-objdump -d of the code object)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ f32x4 chain(int r, f32x4 y0, f32x4 y1) {
    return r == 0 ? y0 : r == 1 ? y0 + y1 : r == 2 ? y0 - y1 : -y1;
}

__global__ void k_chain_uniform(const f32x4* __restrict__ y, f32x4* __restrict__ out, int n) {
    const int r = blockIdx.y >> 2;   // 0..3, 4 blocks in y per r (as xi = 4 r + q)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[(size_t)blockIdx.y * n + i] = chain(r, y[2 * i], y[2 * i + 1]);
}

__global__ void k_chain_lane(const f32x4* __restrict__ y, const int* __restrict__ rr, f32x4* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = chain(rr[i], y[2 * i], y[2 * i + 1]);
}

// the staged form: per thread two tiles, each p[bb] from the chain over (y0, y1) of column bb,
// then m = the same chain over (p[0], p[1]) with q, written to LDS and copied out
__global__ void __launch_bounds__(512) k_chain_staged(const f32x4* __restrict__ y, f32x4* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float ds[16 * 272];
    const int xi = blockIdx.y, r = xi >> 2, q = xi & 3, tid = threadIdx.x;
    const int c4 = (tid & 63) * 4, tp = tid >> 6;
    f32x4 yv[2][2][2];
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int bb = 0; bb < 2; bb++) yv[u][a][bb] = y[(((2 * tp + u) * 2 + a) * 2 + bb) * 64 + (tid & 63)];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const int t = 2 * tp + u;
        f32x4 p[2];
#pragma unroll
        for (int bb = 0; bb < 2; bb++) p[bb] = chain(r, yv[u][0][bb], yv[u][1][bb]);
        const f32x4 m = chain(q, p[0], p[1]);
        *reinterpret_cast<f32x4*>(ds + t * 272 + c4) = m;
    }
    __syncthreads();
    for (int e = tid; e < 16 * 64; e += 512)
        out[(size_t)xi * 16 * 64 + e] = *reinterpret_cast<const f32x4*>(ds + (e >> 6) * 272 + 4 * (e & 63));
}

// the staged form inside a loop over boards with the next board's loads in flight (the
// original's software pipeline): the context in which the original kernel lost the r == 3 arm
__global__ void __launch_bounds__(512) k_chain_loop(const f32x4* __restrict__ y, int nboards, f32x4* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float ds[16 * 272];
    const int xi = blockIdx.y, r = xi >> 2, q = xi & 3, tid = threadIdx.x;
    const int c4 = (tid & 63) * 4, tp = tid >> 6;
    f32x4 yv[2][2][2], acc = f32x4{0.f, 0.f, 0.f, 0.f};
    auto fetch = [&](int b) {
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int bb = 0; bb < 2; bb++)
                    yv[u][a][bb] = y[(size_t)b * 512 + (((2 * tp + u) * 2 + a) * 2 + bb) * 64 + (tid & 63)];
    };
    fetch(0);
    for (int b = 0; b < nboards; b++) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int t = 2 * tp + u;
            f32x4 p[2];
#pragma unroll
            for (int bb = 0; bb < 2; bb++) p[bb] = chain(r, yv[u][0][bb], yv[u][1][bb]);
            const f32x4 m = chain(q, p[0], p[1]);
            *reinterpret_cast<f32x4*>(ds + t * 272 + c4) = m;
        }
        __syncthreads();
        if (b + 1 < nboards) fetch(b + 1);
        acc += *reinterpret_cast<const f32x4*>(ds + (tid >> 5) * 272 + 4 * (tid & 31));
        if (b == 0)
            for (int e = tid; e < 16 * 64; e += 512)
                out[(size_t)xi * 16 * 64 + e] = *reinterpret_cast<const f32x4*>(ds + (e >> 6) * 272 + 4 * (e & 63));
    }
    out[16 * 16 * 64 + (size_t)xi * 512 + tid] = acc;
}

static f32x4 host_chain(int r, f32x4 a, f32x4 b) {
    f32x4 o;
    for (int k = 0; k < 4; k++) o[k] = r == 0 ? a[k] : r == 1 ? a[k] + b[k] : r == 2 ? a[k] - b[k] : -b[k];
    return o;
}
static bool same(f32x4 a, f32x4 b) {
    for (int k = 0; k < 4; k++)
        if (a[k] != b[k]) return false;
    return true;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } } while (0)

int main() {
    const int n = 1 << 16;
    std::vector<f32x4> hy(2 * (size_t)n);
    std::vector<int> hr(n);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xFFFF) / 4096.0f - 8.0f; };
    for (auto& v : hy) v = f32x4{rnd(), rnd(), rnd(), rnd()};
    for (int i = 0; i < n; i++) hr[i] = (i * 7 + i / 64) & 3;
    f32x4 *dy, *dout;
    int* drr;
    CK(hipMalloc(&dy, hy.size() * sizeof(f32x4)));
    CK(hipMalloc(&dout, (size_t)16 * n * sizeof(f32x4)));
    CK(hipMalloc(&drr, n * sizeof(int)));
    CK(hipMemcpy(dy, hy.data(), hy.size() * sizeof(f32x4), hipMemcpyHostToDevice));
    CK(hipMemcpy(drr, hr.data(), n * sizeof(int), hipMemcpyHostToDevice));
    std::vector<f32x4> ho((size_t)16 * n);
    int bad_total = 0;

    // 1. uniform r
    k_chain_uniform<<<dim3(n / 256, 16), 256>>>(dy, dout, n);
    CK(hipGetLastError());
    CK(hipMemcpy(ho.data(), dout, (size_t)16 * n * sizeof(f32x4), hipMemcpyDeviceToHost));
    int bad[4] = {0, 0, 0, 0};
    for (int yb = 0; yb < 16; yb++)
        for (int i = 0; i < n; i++)
            if (!same(ho[(size_t)yb * n + i], host_chain(yb >> 2, hy[2 * i], hy[2 * i + 1]))) bad[yb >> 2]++;
    printf("k_chain_uniform: mismatches per r = %d %d %d %d (of %d each)\n", bad[0], bad[1], bad[2], bad[3], 4 * n);
    bad_total += bad[0] + bad[1] + bad[2] + bad[3];

    // 2. per-lane r
    k_chain_lane<<<n / 256, 256>>>(dy, drr, dout, n);
    CK(hipGetLastError());
    CK(hipMemcpy(ho.data(), dout, (size_t)n * sizeof(f32x4), hipMemcpyDeviceToHost));
    int badl[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++)
        if (!same(ho[i], host_chain(hr[i], hy[2 * i], hy[2 * i + 1]))) badl[hr[i]]++;
    printf("k_chain_lane:    mismatches per r = %d %d %d %d\n", badl[0], badl[1], badl[2], badl[3]);
    bad_total += badl[0] + badl[1] + badl[2] + badl[3];

    // 3. the staged two-level form (r, q) of the weight grad's M' staging
    k_chain_staged<<<dim3(1, 16), 512>>>(dy, dout);
    CK(hipGetLastError());
    CK(hipMemcpy(ho.data(), dout, (size_t)16 * 16 * 64 * sizeof(f32x4), hipMemcpyDeviceToHost));
    int bads[16] = {0};
    for (int xi = 0; xi < 16; xi++)
        for (int t = 0; t < 16; t++)
            for (int l = 0; l < 64; l++) {
                f32x4 p[2];
                for (int bb = 0; bb < 2; bb++)
                    p[bb] = host_chain(xi >> 2, hy[((t * 2 + 0) * 2 + bb) * 64 + l], hy[((t * 2 + 1) * 2 + bb) * 64 + l]);
                if (!same(ho[(size_t)xi * 1024 + t * 64 + l], host_chain(xi & 3, p[0], p[1]))) bads[xi]++;
            }
    printf("k_chain_staged:  mismatches per point xi = 4 r + q:");
    for (int xi = 0; xi < 16; xi++) { printf(" %d", bads[xi]); bad_total += bads[xi]; }
    printf("\n");

    // 4. the staged form inside the software-pipelined board loop (8 boards)
    const int nb = 8;
    k_chain_loop<<<dim3(1, 16), 512>>>(dy, nb, dout);
    CK(hipGetLastError());
    CK(hipMemcpy(ho.data(), dout, (size_t)16 * 16 * 64 * sizeof(f32x4), hipMemcpyDeviceToHost));
    int badp[16] = {0};
    for (int xi = 0; xi < 16; xi++)
        for (int t = 0; t < 16; t++)
            for (int l = 0; l < 64; l++) {
                f32x4 p[2];
                for (int bb = 0; bb < 2; bb++)
                    p[bb] = host_chain(xi >> 2, hy[((t * 2 + 0) * 2 + bb) * 64 + l], hy[((t * 2 + 1) * 2 + bb) * 64 + l]);
                if (!same(ho[(size_t)xi * 1024 + t * 64 + l], host_chain(xi & 3, p[0], p[1]))) badp[xi]++;
            }
    printf("k_chain_loop:    mismatches per point xi = 4 r + q:");
    for (int xi = 0; xi < 16; xi++) { printf(" %d", badp[xi]); bad_total += badp[xi]; }
    printf("\n%s\n", bad_total ? "MISMATCH: the select chain computes wrong values on this GPU" : "all correct");
    return bad_total ? 1 : 0;
}

// mfma_coissue.hip -- how much VALU / LDS-read issue fits beside v_mfma_f32_16x16x4_f32 on gfx950
// (design input for the f32 Winograd tower: DESIGN.md section 5.4).  Per wave: ITER iterations of
// 8 independent MFMAs (8 accumulators) plus NV v_add_f32 (4 independent chains) and ND ds_read_b32
// per iteration.  AG: the accumulators in AccVGPRs (inline-asm MFMA with "+a") instead of ArchVGPRs
// ("+v").  Grid: one workgroup per CU, WPS waves per SIMD.  Reports cycles per MFMA (the
// issue floor is 32) from hipEvent time and the device clock (s_memtime delta per wave).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_coissue tools/mfma_coissue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int NV, int ND, int AG>
__global__ void __launch_bounds__(512) k(float* out, unsigned long long* cyc, int iters) {
    __shared__ float lds[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = (float)i;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    f32x4 acc[8];
    for (int i = 0; i < 8; i++) acc[i] = f32x4{0.f, 0.f, 0.f, (float)lane};
    float a = lane * 1e-3f, b = 1.0f - lane * 1e-3f;
    float v[4] = {a, b, a + b, a - b};
    float d = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int m = 0; m < 8; m++) {
            if constexpr (AG == 1) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc[m]) : "v"(a), "v"(b));
            else if constexpr (AG == 2) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc[m]) : "v"(a), "v"(b));
            else acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NV / 8; j++) v[j & 3] = v[j & 3] + 1.0001f;
#pragma unroll
            for (int j = 0; j < ND / 8; j++) d += lds[(lane * 33 + it * 7 + m * 3 + j * 64) & 4095];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = d + v[0] + v[1] + v[2] + v[3];
    for (int i = 0; i < 8; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int NV, int ND, int AG = 0>
void run(int wps, int iters, float* out, unsigned long long* cyc) {
    const int threads = 256 * wps, grid = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<NV, ND, AG><<<grid, threads>>>(out, cyc, iters / 10);   // warm-up
    hipEventRecord(e0);
    k<NV, ND, AG><<<grid, threads>>>(out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long* h = (unsigned long long*)malloc(grid * 8 * 8);
    hipMemcpy(h, cyc, grid * 8 * 8, hipMemcpyDeviceToHost);
    double c = 0;
    int n = 0;
    for (int i = 0; i < grid * 8; i++)
        if (i % 8 < 4 * wps) { c += h[i]; n++; }
    c /= n;
    const double mfma_per_simd = 8.0 * iters * wps;
    printf("%s  waves/SIMD %d  VALU/MFMA %5.2f  DSread/MFMA %5.2f : %6.2f cycles per MFMA per SIMD (s_memtime), %.3f ms, "
           "%.1f TFLOP/s\n", AG == 1 ? "acc AGPR(asm)" : AG == 2 ? "acc VGPR(asm)" : "acc VGPR    ", wps, NV / 8.0, ND / 8.0, c / mfma_per_simd, ms,
           mfma_per_simd * 4 * 256 * 2048.0 / (ms * 1e-3) / 1e12);
    free(h);
}

int main() {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&cyc, 256 * 8 * 8);
    const int iters = 20000;
    for (int wps = 1; wps <= 2; wps++) {
        run<0, 0>(wps, iters, out, cyc);
        run<8, 0>(wps, iters, out, cyc);
        run<16, 0>(wps, iters, out, cyc);
        run<32, 0>(wps, iters, out, cyc);
        run<0, 0, 2>(wps, iters, out, cyc);
        run<8, 0, 2>(wps, iters, out, cyc);
        run<16, 0, 2>(wps, iters, out, cyc);
        run<32, 0, 2>(wps, iters, out, cyc);
        run<0, 0, 1>(wps, iters, out, cyc);
        run<8, 0, 1>(wps, iters, out, cyc);
        run<16, 0, 1>(wps, iters, out, cyc);
        run<32, 0, 1>(wps, iters, out, cyc);
        run<0, 8, 1>(wps, iters, out, cyc);
        run<8, 8, 1>(wps, iters, out, cyc);
    }
    return 0;
}

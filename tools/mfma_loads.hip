// mfma_loads.hip -- the Winograd tower's inner step in isolation (design input):
// per step 8 v_mfma_f32_16x16x4_f32 (2 accumulator chains x 4 k-slices, as wino_core issues them),
// NW buffer_load_dwordx4 weight fragments into a PF-step register ring and NB ds_read_b128
// B fragments into an LA-step ring, each consumed as the MFMA operands PF / LA steps later.
// Weights stream through a WBYTES buffer (16 KB: L1-resident; 4 MB: one conv's weights, from L2).
// One workgroup per CU, WPS waves per SIMD.  Reports shader cycles per step per wave and per SIMD
// (the MFMA floor is 8 x 32 = 256 cycles per step of one wave).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_loads tools/mfma_loads.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int NW, int NB, int AG, int SOLO = 0>
__global__ void __launch_bounds__(512) k(const float* __restrict__ wts, unsigned wbytes, float* out,
                                         unsigned long long* cyc, int steps) {
    __shared__ __attribute__((aligned(16))) float lds[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = (float)(i & 255) * 1e-3f;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)wts, (short)0, (int)wbytes, 0x00020000);
    const int voff = (w * 2 * 64 + lane) * 16;                  // this wave's 2 fragments of a 16 KB step
    const unsigned nsteps_buf = wbytes / 16384;
    f32x4 acc[16][2];
    for (int x = 0; x < 16; x++)
        for (int n = 0; n < 2; n++) acc[x][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int PF = 2, LA = 4;
    f32x4 wr[PF][2], bq[LA];
    for (int i = 0; i < PF; i++)
        for (int n = 0; n < 2; n++) wr[i][n] = f32x4{1.f, 1.f, 1.f, 1.f};
    const char* lb = reinterpret_cast<const char*>(lds) + lane * 16;
    for (int i = 0; i < LA; i++) bq[i] = *reinterpret_cast<const f32x4*>(lb + i * 1024);
    unsigned soff = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < steps; it += 16) {
#pragma unroll
        for (int st = 0; st < 16; st++) {
            f32x4 a[2] = {wr[st % PF][0], wr[st % PF][1]};
            f32x4 B = bq[st % LA];
            if constexpr (NB > 0) bq[st % LA] = *reinterpret_cast<const f32x4*>(lb + ((st + LA) % 8) * 1024);
            if constexpr (NW > 0) {
#pragma unroll
                for (int n = 0; n < NW; n++)
                    wr[st % PF][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + n * 1024, soff, 0));
                soff = soff + 16384 >= nsteps_buf * 16384 ? 0 : soff + 16384;
            }
            __builtin_amdgcn_sched_barrier(0);
            if (!SOLO || w < 4)
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int n = 0; n < 2; n++) {
                    if constexpr (AG)
                        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc[st][n]) : "v"(a[n][s4]), "v"(B[s4]));
                    else
                        acc[st][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[n][s4], B[s4], acc[st][n], 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int x = 0; x < 16; x++)
        for (int n = 0; n < 2; n++) s += acc[x][n][0] + acc[x][n][3];
    for (int i = 0; i < PF; i++) s += wr[i][0][0] + wr[i][1][1];
    for (int i = 0; i < LA; i++) s += bq[i][2];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int NW, int NB, int AG = 0, int SOLO = 0>
void run(int wps, int steps, const float* wts, unsigned wbytes, float* out, unsigned long long* cyc) {
    const int threads = 256 * wps, grid = 256;
    k<NW, NB, AG, SOLO><<<grid, threads>>>(wts, wbytes, out, cyc, steps / 8);   // warm-up
    k<NW, NB, AG, SOLO><<<grid, threads>>>(wts, wbytes, out, cyc, steps);
    hipDeviceSynchronize();
    unsigned long long h[256 * 8];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    // waves 0-3 (older) and 4-7 (younger, same SIMDs): mean elapsed cycles per step of each half;
    // the SIMD's time is the younger's elapsed (they start together, the older issues first)
    double c0 = 0, c1 = 0;
    for (int b = 0; b < 256; b++)
        for (int i = 0; i < 4; i++) { c0 += h[b * 8 + i]; c1 += wps > 1 ? h[b * 8 + 4 + i] : h[b * 8 + i]; }
    c0 /= 1024.0 * steps;
    c1 /= 1024.0 * steps;
    const double simd = c0 > c1 ? c0 : c1;
    const double mf = SOLO ? 256.0 : 256.0 * wps;
    printf("waves/SIMD %d%s  weights %8u B  %s  buffer_load/step %d  ds_read_b128/step %d : older %6.1f younger %6.1f "
           "cycles/step; SIMD %6.1f cycles per %4.0f MFMA cycles = %.1f %%\n", wps, SOLO ? " (younger: loads only)" : "", wbytes,
           AG ? "acc AGPR" : "acc VGPR", NW, NB, c0, c1, simd, mf, 100.0 * mf / simd);
}

int main() {
    float* out;
    float* wts;
    unsigned long long* cyc;
    const unsigned big = 4u << 20;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&wts, big);
    hipMemset(wts, 0, big);
    hipMalloc(&cyc, 256 * 8 * 8);
    const int steps = 16 * 2000;
    for (int wps = 1; wps <= 2; wps++) {
        run<0, 0>(wps, steps, wts, big, out, cyc);
        run<0, 1>(wps, steps, wts, big, out, cyc);
        run<2, 0>(wps, steps, wts, 16384, out, cyc);
        run<2, 0>(wps, steps, wts, big, out, cyc);
        run<2, 1>(wps, steps, wts, 16384, out, cyc);
        run<2, 1>(wps, steps, wts, big, out, cyc);
        run<2, 1, 1>(wps, steps, wts, 16384, out, cyc);
        run<2, 1, 1>(wps, steps, wts, big, out, cyc);
    }
    run<2, 1, 0, 1>(2, steps, wts, big, out, cyc);
    run<2, 1, 0, 1>(2, steps, wts, 16384, out, cyc);
    return 0;
}

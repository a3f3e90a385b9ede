// wgrad_check.hip -- the fused-transform wino_wgrad_gemm_kernel of tools/wgrad_fused.patch (apply it
// first) against wino_wgrad_transform_kernel +
// a host GEMM on B boards of random data (debug harness).
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off -I alphazero-chess_amd/csrc -o tools/wgrad_check tools/wgrad_check.hip -lrccl
#include "../alphazero-chess_amd/csrc/train.hip"
#include <vector>
int main() {
    const int B = 2, F = 256, K = B * 16;
    std::vector<float> hx((size_t)B * 64 * F), hd((size_t)B * 64 * F);
    unsigned s = 1;
    for (auto& v : hx) { s = s * 1664525u + 1013904223u; v = (float)((s >> 8) & 0xffff) / 65536.f - 0.5f; }
    for (auto& v : hd) { s = s * 1664525u + 1013904223u; v = (float)((s >> 8) & 0xffff) / 65536.f - 0.5f; }
    float *x, *d, *vt, *mt, *part;
    hipMalloc(&x, hx.size() * 4); hipMalloc(&d, hd.size() * 4);
    hipMalloc(&vt, (size_t)16 * K * F * 4); hipMalloc(&mt, (size_t)16 * K * F * 4); hipMalloc(&part, (size_t)16 * F * F * 4);
    hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d, hd.data(), hd.size() * 4, hipMemcpyHostToDevice);
    azi::tr::wino_wgrad_transform_kernel<<<64, 256>>>(x, d, F, B, vt, mt);
    azi::tr::wino_wgrad_gemm_kernel<<<dim3(1, 16), 512>>>(x, d, K, 512, part);
    hipDeviceSynchronize();
    std::vector<float> hv((size_t)16 * K * F), hm((size_t)16 * K * F), hp((size_t)16 * F * F);
    hipMemcpy(hv.data(), vt, hv.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hm.data(), mt, hm.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hp.data(), part, hp.size() * 4, hipMemcpyDeviceToHost);
    double maxerr = 0, maxref = 0; int shown = 0;
    for (int xi = 0; xi < 16; xi++)
        for (int ci = 0; ci < F; ci++)
            for (int co = 0; co < F; co++) {
                double r = 0;
                for (int k = 0; k < K; k++) r += (double)hv[((size_t)xi * K + k) * F + ci] * hm[((size_t)xi * K + k) * F + co];
                const double g = hp[((size_t)xi * F + ci) * F + co], e = fabs(g - r);
                if (e > maxerr) maxerr = e;
                if (fabs(r) > maxref) maxref = fabs(r);
                if (e > 1e-3 && shown < 8) { printf("xi %d ci %d co %d gpu %g ref %g\n", xi, ci, co, g, r); shown++; }
            }
    printf("max err %g (max |ref| %g)\n", maxerr, maxref);
    return maxerr < 1e-3 ? 0 : 1;
}

// detmath.h -- counter-based RNG and bit-reproducible float math for the search.
//
// The reference draws Dirichlet noise (tree.rs:272-289; rand_distr 0.4.3 Dirichlet /
// Gamma) and samples moves (training.rs:318-321; rand 0.8.5 WeightedIndex) from
// thread_rng(), which is not reproducible.  The engine keys a SplitMix64 stream by
// (seed, game, ply, purpose) and evaluates log/exp with the FreeBSD logf/expf
// algorithms written in plain IEEE operations (compiled with -ffp-contract=off), so the
// GPU's noise is identical bit for bit on every run and checkable.
// Gamma(shape<1) = GammaLargeShape(shape+1) * U^(1/shape); large shape by the
// Marsaglia-Tsang squeeze (rand_distr 0.4.3); Dirichlet x_i = g_i * (1/sum g).
#pragma once
#include "chess.h"

#pragma clang fp contract(off)

namespace azc {

AZ_HD uint64_t stream_key(uint64_t seed, uint64_t game, uint64_t ply, uint64_t purpose) {
    uint64_t k = splitmix64(seed ^ 0xA5A5A5A5DEADBEEFULL);
    k = splitmix64(k ^ game);
    return splitmix64(k ^ (ply * 4 + purpose));
}
AZ_HD uint64_t rng_draw(uint64_t key, uint64_t& ctr) {
    uint64_t r = splitmix64(key + ctr * 0xD1B54A32D192ED03ULL);
    ctr++;
    return r;
}
AZ_HD float uniform01(uint64_t key, uint64_t& ctr) { return (float)(rng_draw(key, ctr) >> 40) * 0x1p-24f; }
AZ_HD float open01(uint64_t key, uint64_t& ctr) { return ((float)(rng_draw(key, ctr) >> 41) + 0.5f) * 0x1p-23f; }

AZ_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
AZ_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

AZ_HD float det_logf(float x) {   // FreeBSD e_logf.c, finite x > 0
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    const float Lg1 = 0.66666662693f, Lg2 = 0.40000972152f, Lg3 = 0.28498786688f, Lg4 = 0.24279078841f;
    if (!(x > 0.0f)) return x == 0.0f ? -__builtin_inff() : __builtin_nanf("");
    int32_t k = 0;
    uint32_t ix = f2u(x);
    if (ix < 0x00800000u) { x = x * 0x1p25f; k -= 25; ix = f2u(x); }
    if (ix >= 0x7f800000u) return x;
    k += (int32_t)(ix >> 23) - 127;
    ix &= 0x007fffffu;
    uint32_t i = (ix + (0x95f64u << 3)) & 0x800000u;
    x = u2f(ix | (i ^ 0x3f800000u));
    k += (int32_t)(i >> 23);
    float f = x - 1.0f;
    float s = f / (2.0f + f);
    float z = s * s;
    float w = z * z;
    float t1 = w * (Lg2 + w * Lg4);
    float t2 = z * (Lg1 + w * Lg3);
    float R = t2 + t1;
    float hfsq = 0.5f * f * f;
    float dk = (float)k;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

AZ_HD float det_expf(float x) {   // FreeBSD e_expf.c
    const float o_threshold = 8.8721679688e+01f, u_threshold = -1.0397208405e+02f;
    const float ln2HI = 6.9314575195e-01f, ln2LO = 1.4286067653e-06f, invln2 = 1.4426950216e+00f;
    const float P1 = 1.6666625440e-1f, P2 = -2.7667332906e-3f;
    uint32_t hx = f2u(x);
    int xsb = (int)(hx >> 31);
    hx &= 0x7fffffffu;
    float hi = 0.0f, lo = 0.0f;
    int32_t k = 0;
    if (hx >= 0x42b17218u) {
        if (hx > 0x7f800000u) return x + x;
        if (hx == 0x7f800000u) return xsb == 0 ? x : 0.0f;
        if (x > o_threshold) return __builtin_inff();
        if (x < u_threshold) return 0.0f;
    }
    if (hx > 0x3eb17218u) {
        if (hx < 0x3F851592u) {
            hi = x - (xsb ? -ln2HI : ln2HI);
            lo = xsb ? -ln2LO : ln2LO;
            k = 1 - xsb - xsb;
        } else {
            k = (int32_t)(invln2 * x + (xsb ? -0.5f : 0.5f));
            float t = (float)k;
            hi = x - t * ln2HI;
            lo = t * ln2LO;
        }
        x = hi - lo;
    } else if (hx < 0x39000000u) {
        return 1.0f + x;
    } else {
        k = 0;
    }
    float t = x * x;
    float twopk = k >= -125 ? u2f((uint32_t)(0x7f + k) << 23) : u2f((uint32_t)(0x7f + (k + 100)) << 23);
    float c = x - t * (P1 + t * P2);
    if (k == 0) return 1.0f - ((x * c) / (c - 2.0f) - x);
    float y = 1.0f - ((lo - (x * c) / (2.0f - c)) - hi);
    if (k >= -125) {
        if (k == 128) return y * 2.0f * 0x1p127f;
        return y * twopk;
    }
    return y * twopk * 0x1p-100f;
}

AZ_HD float std_normal(uint64_t key, uint64_t& ctr) {   // Marsaglia polar
    for (;;) {
        float u = 2.0f * uniform01(key, ctr) - 1.0f;
        float v = 2.0f * uniform01(key, ctr) - 1.0f;
        float s = u * u + v * v;
        if (s >= 1.0f || s == 0.0f) continue;
        return u * sqrtf(-2.0f * det_logf(s) / s);
    }
}

AZ_HD float gamma_large(float shape, uint64_t key, uint64_t& ctr) {
    float d = shape - 1.0f / 3.0f;
    float c = 1.0f / sqrtf(9.0f * d);
    for (;;) {
        float x = std_normal(key, ctr);
        float v_cbrt = 1.0f + c * x;
        if (v_cbrt <= 0.0f) continue;
        float v = v_cbrt * v_cbrt * v_cbrt;
        float u = open01(key, ctr);
        float x_sqr = x * x;
        if (u < 1.0f - 0.0331f * x_sqr * x_sqr || det_logf(u) < 0.5f * x_sqr + d * (1.0f - v + det_logf(v)))
            return d * v;
    }
}

AZ_HD float gamma_sample(float shape, uint64_t key) {
    uint64_t ctr = 0;
    if (shape < 1.0f) {
        float inv_shape = 1.0f / shape;
        float u = open01(key, ctr);
        float g = gamma_large(shape + 1.0f, key, ctr);
        return g * det_expf(det_logf(u) * inv_shape);
    }
    return gamma_large(shape, key, ctr);
}

AZ_HD uint64_t dirichlet_component_key(uint64_t key, int i) {
    return splitmix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
}

}  // namespace azc

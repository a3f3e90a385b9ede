/*
 * detrng_ref.c -- ORACLE (test infrastructure only, see az_oracle.h).
 *
 * The reference draws its Dirichlet noise (tree.rs:272-289, rand_distr 0.4.3
 * Dirichlet/Gamma) and its move samples (training.rs:318-321, rand 0.8.5
 * WeightedIndex) from thread_rng(), which is OS-seeded and not reproducible
 * (SURVEY 0).  The build replaces that stream with a counter-based one
 * (SplitMix64 keyed by seed/game/ply/purpose) and uses only IEEE basic operations
 * (+ - * / sqrt, no contraction) plus the FreeBSD logf/expf algorithms written out
 * below, so the CPU oracle and the GPU path draw bit-identical noise.
 * The sampling algorithms follow rand_distr 0.4.3:
 *   Gamma(shape<1): GammaSmallShape = GammaLargeShape(shape+1) * U^(1/shape)
 *   GammaLargeShape: Marsaglia-Tsang squeeze with a standard normal
 *   Dirichlet: g_i ~ Gamma(alpha_i), x_i = g_i * (1 / sum g)
 * (the standard normal is drawn by the Marsaglia polar method, not rand_distr's
 * ziggurat; the stream is ours either way).
 */
#include "az_oracle.h"
#include <math.h>
#include <string.h>

uint64_t ref_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

uint64_t ref_stream_key(uint64_t seed, uint64_t game, uint64_t ply, uint64_t purpose) {
    uint64_t k = ref_splitmix64(seed ^ 0xA5A5A5A5DEADBEEFULL);
    k = ref_splitmix64(k ^ game);
    return ref_splitmix64(k ^ (ply * 4 + purpose));
}

static uint64_t draw(uint64_t key, uint64_t* ctr) {
    uint64_t r = ref_splitmix64(key + (*ctr) * 0xD1B54A32D192ED03ULL);
    (*ctr)++;
    return r;
}

float ref_uniform01(uint64_t key, uint64_t* ctr) {      /* [0,1), 24-bit */
    return (float)(draw(key, ctr) >> 40) * 0x1p-24f;
}

float ref_open01(uint64_t key, uint64_t* ctr) {         /* (0,1) */
    return ((float)(draw(key, ctr) >> 41) + 0.5f) * 0x1p-23f;
}

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* FreeBSD e_logf.c, for finite x > 0 */
float ref_det_logf(float x) {
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    const float Lg1 = 0.66666662693f, Lg2 = 0.40000972152f, Lg3 = 0.28498786688f, Lg4 = 0.24279078841f;
    if (!(x > 0.0f)) return x == 0.0f ? -INFINITY : NAN;
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

/* FreeBSD e_expf.c */
float ref_det_expf(float x) {
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
        if (x > o_threshold) return INFINITY;
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
    float twopk;
    if (k >= -125) twopk = u2f((uint32_t)(0x7f + k) << 23);
    else twopk = u2f((uint32_t)(0x7f + (k + 100)) << 23);
    float c = x - t * (P1 + t * P2);
    if (k == 0) return 1.0f - ((x * c) / (c - 2.0f) - x);
    float y = 1.0f - ((lo - (x * c) / (2.0f - c)) - hi);
    if (k >= -125) {
        if (k == 128) return y * 2.0f * 0x1p127f;
        return y * twopk;
    }
    return y * twopk * 0x1p-100f;
}

static float std_normal(uint64_t key, uint64_t* ctr) {   /* Marsaglia polar */
    for (;;) {
        float u = 2.0f * ref_uniform01(key, ctr) - 1.0f;
        float v = 2.0f * ref_uniform01(key, ctr) - 1.0f;
        float s = u * u + v * v;
        if (s >= 1.0f || s == 0.0f) continue;
        return u * sqrtf(-2.0f * ref_det_logf(s) / s);
    }
}

static float gamma_large(float shape, uint64_t key, uint64_t* ctr) {
    float d = shape - 1.0f / 3.0f;
    float c = 1.0f / sqrtf(9.0f * d);
    for (;;) {
        float x = std_normal(key, ctr);
        float v_cbrt = 1.0f + c * x;
        if (v_cbrt <= 0.0f) continue;
        float v = v_cbrt * v_cbrt * v_cbrt;
        float u = ref_open01(key, ctr);
        float x_sqr = x * x;
        if (u < 1.0f - 0.0331f * x_sqr * x_sqr ||
            ref_det_logf(u) < 0.5f * x_sqr + d * (1.0f - v + ref_det_logf(v)))
            return d * v;
    }
}

float ref_gamma(float shape, uint64_t key) {
    uint64_t ctr = 0;
    if (shape < 1.0f) {
        float inv_shape = 1.0f / shape;
        float u = ref_open01(key, &ctr);
        float g = gamma_large(shape + 1.0f, key, &ctr);
        return g * ref_det_expf(ref_det_logf(u) * inv_shape);
    }
    return gamma_large(shape, key, &ctr);
}

void ref_dirichlet(float alpha, int n, uint64_t key, float* out) {
    float sum = 0.0f;
    for (int i = 0; i < n; i++) {
        out[i] = ref_gamma(alpha, ref_splitmix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL));
        sum = sum + out[i];
    }
    float invacc = 1.0f / sum;
    for (int i = 0; i < n; i++) out[i] = out[i] * invacc;
}

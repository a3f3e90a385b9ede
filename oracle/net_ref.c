/*
 * net_ref.c -- ORACLE (test infrastructure only, see az_oracle.h).
 *
 * fp32 restatement of AlphaZero::forward (agent.rs:112-144) with burn 0.18 inference
 * semantics: Conv2d 3x3 "same" padding with bias, BatchNorm from running stats
 * ((x - mean) / sqrt(var + 1e-5) * gamma + beta, burn BatchNorm::forward in
 * inference mode), ReLU, residual blocks (agent.rs:33-45), policy head
 * 1x1 F->32, BN, ReLU, 1x1 32->64, reshape [N,4096] (index c*64+h*8+w), softmax
 * (agent.rs:124-130), value head 1x1 F->8, BN, ReLU, flatten 512, Linear 512->64,
 * ReLU, Linear 64->1, tanh (agent.rs:133-141).  BN is NOT folded here (the product
 * folds it at load time; the difference is inside the stated tolerance).
 *
 * Flat parameter layout (shared with include/az.h, az_net_create):
 *   input_conv.weight [F,19,3,3]  input_conv.bias [F]  input_bn {gamma,beta,mean,var}[F]
 *   per block: conv1.weight [F,F,3,3] conv1.bias [F] bn1{4}[F] conv2.weight conv2.bias bn2{4}
 *   policy_conv_1.weight [32,F] .bias [32] policy_bn{4}[32]
 *   policy_conv_2.weight [64,32] .bias [64]
 *   value_conv.weight [8,F] .bias [8] value_bn{4}[8]
 *   value_linear_1.weight [512,64] (burn Linear layout [d_in, d_out]) .bias [64]
 *   value_linear_2.weight [64,1] .bias [1]
 */
#include "az_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

struct ref_net {
    int blocks, filters;
    float* w;                 /* flat copy */
    const float *in_w, *in_b, *in_bn;
    const float **c1w, **c1b, **bn1, **c2w, **c2b, **bn2;
    const float *p1w, *p1b, *pbn, *p2w, *p2b;
    const float *vw, *vb, *vbn, *l1w, *l1b, *l2w, *l2b;
};

size_t ref_net_num_params(int B, int F) {
    size_t n = (size_t)F * 19 * 9 + F + 4 * (size_t)F;
    n += (size_t)B * 2 * ((size_t)F * F * 9 + F + 4 * (size_t)F);
    n += 32 * (size_t)F + 32 + 4 * 32;
    n += 64 * 32 + 64;
    n += 8 * (size_t)F + 8 + 4 * 8;
    n += 512 * 64 + 64 + 64 + 1;
    return n;
}

ref_net* ref_net_create(int B, int F, const float* flat) {
    ref_net* n = (ref_net*)calloc(1, sizeof(ref_net));
    size_t np = ref_net_num_params(B, F);
    n->blocks = B; n->filters = F;
    n->w = (float*)malloc(np * sizeof(float));
    memcpy(n->w, flat, np * sizeof(float));
    n->c1w = calloc((size_t)B + 1, sizeof(float*)); n->c1b = calloc((size_t)B + 1, sizeof(float*));
    n->bn1 = calloc((size_t)B + 1, sizeof(float*)); n->c2w = calloc((size_t)B + 1, sizeof(float*));
    n->c2b = calloc((size_t)B + 1, sizeof(float*)); n->bn2 = calloc((size_t)B + 1, sizeof(float*));
    const float* p = n->w;
    n->in_w = p; p += (size_t)F * 19 * 9;
    n->in_b = p; p += F;
    n->in_bn = p; p += 4 * (size_t)F;
    for (int b = 0; b < B; b++) {
        n->c1w[b] = p; p += (size_t)F * F * 9;
        n->c1b[b] = p; p += F;
        n->bn1[b] = p; p += 4 * (size_t)F;
        n->c2w[b] = p; p += (size_t)F * F * 9;
        n->c2b[b] = p; p += F;
        n->bn2[b] = p; p += 4 * (size_t)F;
    }
    n->p1w = p; p += 32 * (size_t)F;
    n->p1b = p; p += 32;
    n->pbn = p; p += 4 * 32;
    n->p2w = p; p += 64 * 32;
    n->p2b = p; p += 64;
    n->vw = p; p += 8 * (size_t)F;
    n->vb = p; p += 8;
    n->vbn = p; p += 4 * 8;
    n->l1w = p; p += 512 * 64;
    n->l1b = p; p += 64;
    n->l2w = p; p += 64;
    n->l2b = p; p += 1;
    return n;
}

void ref_net_free(ref_net* n) {
    if (!n) return;
    free(n->w); free(n->c1w); free(n->c1b); free(n->bn1); free(n->c2w); free(n->c2b); free(n->bn2);
    free(n);
}

/* out[co][64] = bias[co] + sum_ci sum_tap w[co][ci][tap] * in[ci][shifted]  (NCHW, one board) */
static void conv3x3(const float* in, int cin, const float* w, const float* bias, int cout, float* out) {
    for (int co = 0; co < cout; co++) {
        float acc[64];
        for (int s = 0; s < 64; s++) acc[s] = 0.0f;
        for (int ci = 0; ci < cin; ci++) {
            const float* x = in + ci * 64;
            const float* wk = w + ((size_t)co * cin + ci) * 9;
            for (int kh = 0; kh < 3; kh++) {
                int dr = kh - 1;
                for (int kw = 0; kw < 3; kw++) {
                    int df = kw - 1;
                    float wv = wk[kh * 3 + kw];
                    int r0 = dr < 0 ? 1 : 0, r1 = dr > 0 ? 7 : 8;
                    int f0 = df < 0 ? 1 : 0, f1 = df > 0 ? 7 : 8;
                    for (int r = r0; r < r1; r++) {
                        const float* xr = x + (r + dr) * 8 + df;
                        float* ar = acc + r * 8;
                        for (int f = f0; f < f1; f++) ar[f] += wv * xr[f];
                    }
                }
            }
        }
        for (int s = 0; s < 64; s++) out[co * 64 + s] = acc[s] + bias[co];
    }
}

static void conv1x1(const float* in, int cin, const float* w, const float* bias, int cout, float* out) {
    for (int co = 0; co < cout; co++) {
        float acc[64];
        for (int s = 0; s < 64; s++) acc[s] = 0.0f;
        for (int ci = 0; ci < cin; ci++) {
            float wv = w[co * cin + ci];
            const float* x = in + ci * 64;
            for (int s = 0; s < 64; s++) acc[s] += wv * x[s];
        }
        for (int s = 0; s < 64; s++) out[co * 64 + s] = acc[s] + bias[co];
    }
}

/* burn BatchNorm inference: ((x - mean) / sqrt(var + eps)) * gamma + beta, then optional relu */
static void batchnorm(float* x, int c, const float* bn, int relu) {
    const float *gamma = bn, *beta = bn + c, *mean = bn + 2 * c, *var = bn + 3 * c;
    for (int ch = 0; ch < c; ch++) {
        float sd = sqrtf(var[ch] + 1e-5f);
        for (int s = 0; s < 64; s++) {
            float v = ((x[ch * 64 + s] - mean[ch]) / sd) * gamma[ch] + beta[ch];
            x[ch * 64 + s] = relu ? (v > 0.0f ? v : 0.0f) : v;
        }
    }
}

static void forward_one(const ref_net* n, const float* planes, float* policy, float* value) {
    int F = n->filters;
    float* x = (float*)malloc(sizeof(float) * 64 * (size_t)F);
    float* h = (float*)malloc(sizeof(float) * 64 * (size_t)F);
    float* t = (float*)malloc(sizeof(float) * 64 * (size_t)F);
    conv3x3(planes, 19, n->in_w, n->in_b, F, x);
    batchnorm(x, F, n->in_bn, 1);
    for (int b = 0; b < n->blocks; b++) {
        conv3x3(x, F, n->c1w[b], n->c1b[b], F, h);
        batchnorm(h, F, n->bn1[b], 1);
        conv3x3(h, F, n->c2w[b], n->c2b[b], F, t);
        batchnorm(t, F, n->bn2[b], 0);
        for (int i = 0; i < 64 * F; i++) { float v = t[i] + x[i]; x[i] = v > 0.0f ? v : 0.0f; }
    }
    /* policy head */
    float p1[32 * 64], logits[4096];
    conv1x1(x, F, n->p1w, n->p1b, 32, p1);
    batchnorm(p1, 32, n->pbn, 1);
    conv1x1(p1, 32, n->p2w, n->p2b, 64, logits);
    float m = -INFINITY;
    for (int i = 0; i < 4096; i++) m = logits[i] > m ? logits[i] : m;
    double sum = 0.0;
    for (int i = 0; i < 4096; i++) { float e = expf(logits[i] - m); policy[i] = e; sum += e; }
    float fs = (float)sum;
    for (int i = 0; i < 4096; i++) policy[i] = policy[i] / fs;
    /* value head */
    float v8[8 * 64], hdn[64];
    conv1x1(x, F, n->vw, n->vb, 8, v8);
    batchnorm(v8, 8, n->vbn, 1);
    for (int o = 0; o < 64; o++) {
        float acc = 0.0f;
        for (int i = 0; i < 512; i++) acc += v8[i] * n->l1w[i * 64 + o];
        acc += n->l1b[o];
        hdn[o] = acc > 0.0f ? acc : 0.0f;
    }
    float acc = 0.0f;
    for (int i = 0; i < 64; i++) acc += hdn[i] * n->l2w[i];
    acc += n->l2b[0];
    *value = tanhf(acc);
    free(x); free(h); free(t);
}

void ref_net_forward(const ref_net* n, const float* planes, int batch, float* policy, float* value, int threads) {
    (void)threads;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
    for (int b = 0; b < batch; b++)
        forward_one(n, planes + (size_t)b * 19 * 64, policy + (size_t)b * 4096, value + b);
}

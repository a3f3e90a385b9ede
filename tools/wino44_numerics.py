"""Pricing study (round 6, CPU, numpy): the f32 rounding of Winograd F(2x2,3x3) against F(4x4,3x3) on a
20x256 residual tower of random-init 3x3 convs over 8x8 boards (4 boards; BatchNorm at its random-init
identity, ReLU, residual adds), each against the same tower in float64 with direct convs.  The
transforms and the point GEMMs run in float32 (numpy's f32 einsum / matmul: blocked sums, not the
MFMA's order -- the error scale, not the bits); U = G g G^T in float64, rounded once, as on the GPU.
Cook-Toom matrices from the interpolation points (B^T solved from the bilinear identity).
Usage: python tools/wino44_numerics.py [filters=256] [blocks=20]   (output: profiles/r06_wino44_numerics.txt)"""
import numpy as np, itertools, sys
rng = np.random.default_rng(0)

def cook_toom(m, r, pts):
    n = m + r - 1
    assert len(pts) == n - 1
    AT = np.zeros((m, n)); G = np.zeros((n, r))
    for j, p in enumerate(pts):
        for i in range(m): AT[i, j] = p ** i
        den = np.prod([p - q for q in pts if q != p])
        for k in range(r): G[j, k] = p ** k / den
    AT[m - 1, n - 1] = 1; G[n - 1, r - 1] = 1
    # solve B^T from y_i = sum_j AT[i,j] (G g)_j (BT d)_j
    rows = []; rhs = []
    for trial in range(4 * n):
        g = rng.standard_normal(r); d = rng.standard_normal(n)
        Gg = G @ g
        for i in range(m):
            row = np.zeros((n, n))
            for j in range(n): row[j, :] = AT[i, j] * Gg[j] * d
            rows.append(row.ravel()); rhs.append(sum(g[k] * d[i + k] for k in range(r)))
    BT = np.linalg.lstsq(np.array(rows), np.array(rhs), rcond=None)[0].reshape(n, n)
    BT[np.abs(BT) < 1e-12] = 0
    return AT, G, BT

def conv_direct(x, w, dt):   # x [B,8,8,C], w [Co,Ci,3,3]
    B, H, W, C = x.shape
    xp = np.zeros((B, H + 2, W + 2, C), dt); xp[:, 1:-1, 1:-1] = x
    cols = np.stack([xp[:, i:i + H, j:j + W, :] for i in range(3) for j in range(3)], axis=3)  # B,H,W,9,C
    wm = w.transpose(2, 3, 1, 0).reshape(9 * C, -1).astype(dt)
    return (cols.reshape(B * H * W, 9 * C).astype(dt) @ wm).reshape(B, H, W, -1)

def conv_wino(x, w, m, mats):
    AT, G, BT = mats
    n = m + 2
    B, H, W, C = x.shape
    Co = w.shape[0]
    U = np.einsum('ik,ockl,jl->ijoc', G, w.astype(np.float64), G).astype(np.float32)  # f64 transform, rounded once
    xp = np.zeros((B, H + 2, W + 2, C), np.float32); xp[:, 1:-1, 1:-1] = x
    T = H // m
    out = np.zeros((B, H, W, Co), np.float32)
    BT32 = BT.astype(np.float32); AT32 = AT.astype(np.float32)
    for ty in range(T):
        for tx in range(T):
            d = xp[:, ty * m:ty * m + n, tx * m:tx * m + n, :]             # B,n,n,C
            V = np.einsum('ia,bajc,kj->bikc', BT32, d, BT32).astype(np.float32)  # f32 ops
            M = np.einsum('ijoc,bijc->bijo', U, V).astype(np.float32)
            Y = np.einsum('ai,bijo,cj->baco', AT32, M, AT32).astype(np.float32)
            out[:, ty * m:(ty + 1) * m, tx * m:(tx + 1) * m, :] = Y
    return out

def tower(x, ws, conv, dt):
    eps = 1e-5; s = dt(1.0 / np.sqrt(1.0 + eps))
    h = x
    for b in range(len(ws) // 2):
        y = np.maximum(conv(h, ws[2 * b]) * s, 0).astype(dt)
        y = (conv(y, ws[2 * b + 1]) * s + h).astype(dt)
        h = np.maximum(y, 0).astype(dt)
    return h

F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 20
Bn = 4
bound = 1.0 / np.sqrt(F * 9)
ws = [rng.uniform(-bound, bound, (F, F, 3, 3)) for _ in range(2 * NB)]
x0 = np.maximum(rng.standard_normal((Bn, 8, 8, F)), 0)   # stand-in for the input conv's output
ref = tower(x0, ws, lambda h, w: conv_direct(h, w, np.float64), np.float64)
f32d = tower(x0.astype(np.float32), ws, lambda h, w: conv_direct(h, w.astype(np.float32), np.float32), np.float32)
m22 = cook_toom(2, 3, [0, 1, -1])
m44 = cook_toom(4, 3, [0, 1, -1, 2, -2])
m44h = cook_toom(4, 3, [0, 1, -1, 0.5, -0.5])
res = {}
res['f32 direct'] = f32d
res['F(2x2) 0,+-1'] = tower(x0.astype(np.float32), ws, lambda h, w: conv_wino(h, w, 2, m22), np.float32)
res['F(4x4) 0,+-1,+-2'] = tower(x0.astype(np.float32), ws, lambda h, w: conv_wino(h, w, 4, m44), np.float32)
res['F(4x4) 0,+-1,+-1/2'] = tower(x0.astype(np.float32), ws, lambda h, w: conv_wino(h, w, 4, m44h), np.float32)
sc = np.abs(ref).max()
for k, v in res.items():
    e = np.abs(v - ref)
    # a value-head-like scalar: mean over squares/channels, and a policy-like logit: one channel dot
    vh = v.reshape(Bn, -1).mean(1); rh = ref.reshape(Bn, -1).mean(1)
    print('%-22s max abs err %.3e  rel-to-max %.3e  rms rel %.3e  mean-pool err %.3e' % (k, e.max(), e.max() / sc, np.sqrt((e ** 2).mean() / (ref ** 2).mean()), np.abs(vh - rh).max()))

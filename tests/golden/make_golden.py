"""Generates tests/golden/net_2x32.npz: golden vectors for AlphaZero::forward
(agent.rs:112-144) computed with torch on the CPU of the build container (float64).

The reference (burn 0.18 / CUDA) cannot run here, so torch's conv2d(padding=1) +
batch_norm(eval) + relu / softmax / tanh restates burn's semantics
(Conv2d PaddingConfig2d::Same, BatchNorm inference with running stats, eps 1e-5).
Inputs: 16 positions from seeded random playouts, encoded with the oracle's to_tensor.
Weights: seeded random init (azchess.random_weights layout), stored in the fixture.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as Fn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def split(flat, B, F):
    p = 0
    out = {}

    def take(name, n, shape):
        nonlocal p
        out[name] = torch.tensor(flat[p:p + n], dtype=torch.float64).reshape(shape)
        p += n

    take("in_w", F * 19 * 9, (F, 19, 3, 3)); take("in_b", F, (F,)); take("in_bn", 4 * F, (4, F))
    for b in range(B):
        for k in (1, 2):
            take("c%d_%d_w" % (b, k), F * F * 9, (F, F, 3, 3)); take("c%d_%d_b" % (b, k), F, (F,))
            take("c%d_%d_bn" % (b, k), 4 * F, (4, F))
    take("p1w", 32 * F, (32, F, 1, 1)); take("p1b", 32, (32,)); take("pbn", 128, (4, 32))
    take("p2w", 64 * 32, (64, 32, 1, 1)); take("p2b", 64, (64,))
    take("vw", 8 * F, (8, F, 1, 1)); take("vb", 8, (8,)); take("vbn", 32, (4, 8))
    take("l1w", 512 * 64, (512, 64)); take("l1b", 64, (64,)); take("l2w", 64, (64, 1)); take("l2b", 1, (1,))
    assert p == len(flat)
    return out


def bn(x, t):
    return Fn.batch_norm(x, t[2], t[3], t[0], t[1], training=False, eps=1e-5)


def forward(W, x, B):
    x = Fn.relu(bn(Fn.conv2d(x, W["in_w"], W["in_b"], padding=1), W["in_bn"]))
    for b in range(B):
        h = Fn.relu(bn(Fn.conv2d(x, W["c%d_1_w" % b], W["c%d_1_b" % b], padding=1), W["c%d_1_bn" % b]))
        h = bn(Fn.conv2d(h, W["c%d_2_w" % b], W["c%d_2_b" % b], padding=1), W["c%d_2_bn" % b])
        x = Fn.relu(h + x)
    p = Fn.relu(bn(Fn.conv2d(x, W["p1w"], W["p1b"]), W["pbn"]))
    p = Fn.conv2d(p, W["p2w"], W["p2b"]).reshape(x.shape[0], -1)
    pol = torch.softmax(p, dim=1)
    v = Fn.relu(bn(Fn.conv2d(x, W["vw"], W["vb"]), W["vbn"])).reshape(x.shape[0], -1)
    v = Fn.relu(v @ W["l1w"] + W["l1b"])
    v = torch.tanh(v @ W["l2w"] + W["l2b"]).squeeze(1)
    return pol, v


def random_weights(B, F, seed):
    """Same definition as azchess.agent.random_weights (kept here so the fixture is self-contained)."""
    rng = np.random.default_rng(seed)
    parts = []
    shapes = [((F, 19, 3, 3), 171), ((F,), 171), None]
    for _ in range(B):
        shapes += [((F, F, 3, 3), 9 * F), ((F,), 9 * F), None] * 2
    shapes += [((32, F), F), ((32,), F), None, ((64, 32), 32), ((64,), 32), ((8, F), F), ((8,), F), None,
               ((512, 64), 512), ((64,), 512), ((64, 1), 64), ((1,), 64)]
    bn_c = [F] + [F, F] * B + [32, 8]
    k = 0
    for s in shapes:
        if s is None:
            c = bn_c[k]; k += 1
            parts.append(np.concatenate([1 + 1e-2 * rng.uniform(-1, 1, c), 1e-2 * rng.uniform(-1, 1, c),
                                         1e-2 * rng.uniform(-1, 1, c), 1 + 1e-2 * rng.uniform(-1, 1, c)]))
        else:
            bound = 1.0 / np.sqrt(s[1])
            parts.append(rng.uniform(-bound, bound, int(np.prod(s[0]))))
    return np.concatenate(parts).astype(np.float32)


def positions(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        g = O.Game()
        for ply in range(int(rng.integers(0, 80))):
            idx = O.legal_indices(g.position)
            if len(idx) == 0 or g.play_index(int(rng.choice(idx))) != 0:
                break
        if len(O.legal_indices(g.position)):
            out.append(O.to_tensor(g.position))
    return np.stack(out)


def main():
    B, F = 2, 32
    w = random_weights(B, F, 42)
    assert w.size == O.num_params(B, F)
    planes = positions(16, 3)
    W = split(w.astype(np.float64), B, F)
    with torch.no_grad():
        pol, val = forward(W, torch.tensor(planes, dtype=torch.float64), B)
    np.savez_compressed(os.path.join(HERE, "net_2x32.npz"), weights=w, planes=planes,
                        policy=pol.numpy().astype(np.float32), value=val.numpy().astype(np.float32), blocks=B, filters=F)
    print("wrote net_2x32.npz", planes.shape, float(val.abs().max()))


if __name__ == "__main__":
    main()

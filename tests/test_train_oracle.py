"""CPU pins of the training oracle (oracle/train_ref.py) -- its restatements of burn's
BatchNorm::forward_train and AdamW checked against torch's own implementations where the two
agree mathematically, and get_cyclical_lr against hand-computed values of training.rs:424-441."""
import numpy as np
import pytest
import torch

import azchess as A
import train_ref as T


def test_cyclical_lr_values():
    # base 1e-3, max 1e-2, cycle 20, half 10, decay x0.1 every 1000 iterations
    assert T.cyclical_lr(0) == pytest.approx(1e-3)
    assert T.cyclical_lr(10) == pytest.approx(1e-2)
    assert T.cyclical_lr(5) == pytest.approx(5.5e-3)
    assert T.cyclical_lr(15) == pytest.approx(5.5e-3)
    assert T.cyclical_lr(20) == pytest.approx(1e-3)
    assert T.cyclical_lr(1010) == pytest.approx(1e-3)
    for it in [0, 3, 10, 11, 19, 999, 1000, 2345, 9999]:
        assert A.get_cyclical_lr(it) == T.cyclical_lr(it)   # the C-ABI's restatement, bit-equal


def test_layout_matches_the_product():
    for b, f in [(2, 32), (20, 256)]:
        _, n = T.segments(b, f)
        assert n == A.num_params(b, f)
        assert [s[:2] for s in T.param_shapes(b, f)] == [s[:2] for s in A.agent.param_shapes(b, f)]


def test_batchnorm_restatement_vs_torch():
    rng = np.random.default_rng(0)
    x = torch.tensor(rng.normal(size=(6, 5, 8, 8)), dtype=torch.float64)
    g = torch.tensor(rng.uniform(0.5, 1.5, 5))
    b = torch.tensor(rng.normal(size=5))
    ref = T.TrainRef.__new__(T.TrainRef)
    ref.P = {"bn.gamma": g, "bn.beta": b}
    ref.stats = {"bn": [torch.zeros(5, dtype=torch.float64), torch.ones(5, dtype=torch.float64)]}
    y = ref._bn(x, "bn")
    rm, rv = torch.zeros(5, dtype=torch.float64), torch.ones(5, dtype=torch.float64)
    yt = torch.nn.functional.batch_norm(x, rm, rv, g, b, training=True, momentum=0.1, eps=1e-5)
    assert torch.allclose(y, yt, atol=1e-12)
    assert torch.allclose(ref.stats["bn"][0], rm, atol=1e-15)
    # burn keeps the biased variance; torch's running var is unbiased: v_b = v_u * (n-1)/n
    n = 6 * 64
    vb = x.var(dim=(0, 2, 3), unbiased=False)
    assert torch.allclose(ref.stats["bn"][1], 0.9 + 0.1 * vb, atol=1e-15)
    assert torch.allclose((rv - 0.9) / 0.1 * (n - 1) / n, vb, atol=1e-12)


def test_adamw_restatement_vs_torch_adamw():
    rng = np.random.default_rng(1)
    p0 = rng.normal(size=1000).astype(np.float32)
    mask = np.ones(1000, bool)
    m = np.zeros_like(p0)
    v = np.zeros_like(p0)
    p = p0.copy()
    tp = torch.tensor(p0.astype(np.float64), requires_grad=True)
    opt = torch.optim.AdamW([tp], lr=1e-3, betas=(0.9, 0.999), eps=1e-5, weight_decay=1e-4)
    for step in range(1, 6):
        g = (rng.normal(size=1000) * 0.5).astype(np.float32)
        p, m, v = T.adamw_step(p, g, m, v, mask, step, 1e-3)
        tp.grad = torch.tensor(np.clip(g, -1, 1).astype(np.float64))
        opt.step()
        assert np.allclose(p, tp.detach().numpy(), rtol=0, atol=2e-6)


def test_oracle_gradients_vs_finite_differences():
    blocks, F = 1, 16
    w = A.random_weights(blocks, F, seed=2)
    rng = np.random.default_rng(3)
    planes = (rng.random((3, 19, 64)) < 0.2).astype(np.float32)
    tpol = rng.dirichlet(np.ones(4096) * 0.1, 3).astype(np.float32)
    tval = rng.uniform(-1, 1, 3).astype(np.float32)
    g, _ = T.TrainRef(blocks, F, w).grads(planes, tpol, tval)
    seg, _ = T.segments(blocks, F)

    def loss(flat):
        with torch.no_grad():
            pol, val = T.TrainRef(blocks, F, flat).forward(planes)
        t = torch.tensor(tpol, dtype=torch.float64)
        z = torch.tensor(tval, dtype=torch.float64)
        return float(-(t * torch.log(pol + 1e-5)).sum(1).mean() + 0.5 * ((val - z) ** 2).mean())

    for name in ["res_blocks.0.conv2.weight", "value_linear_1.weight", "policy_conv_2.bias"]:
        o = seg[name][0]
        for k in (0, 7):
            e = w.astype(np.float64).copy()
            h = 1e-3
            e[o + k] += h
            lp = loss(e)
            e[o + k] -= 2 * h
            lm = loss(e)
            fd = (lp - lm) / (2 * h)
            assert abs(fd - g[o + k]) <= 1e-4 * (1 + abs(fd)), (name, k, fd, g[o + k])

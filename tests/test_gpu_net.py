"""HIP network (MFMA conv tower + fused heads) against the torch golden vectors and the
oracle.  Tolerances (stated per north_star "policy/value within a stated fp tolerance"):
  f32 path (v_mfma_f32_16x16x4_f32, exact f32 FMA chains, BN folded):
      value |d| <= 1e-5, policy |d| <= 1e-4 * p + 1e-8
  bf16 path (bf16 weights/activations, f32 accumulate):
      value |d| <= 2e-2, policy |d| <= 5e-2 * p + 2e-5 and total-variation <= 2e-2
"""
import os

import numpy as np
import pytest

import azchess as A
import oracle as O
from conftest import ROOT

pytestmark = pytest.mark.gpu

TOL = {"f32": dict(v=1e-5, prel=1e-4, pabs=1e-8), "bf16": dict(v=2e-2, prel=5e-2, pabs=2e-5)}


def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "net_2x32.npz"))


def check(pol, val, rpol, rval, dtype):
    t = TOL[dtype]
    assert np.all(np.abs(val - rval) <= t["v"]), np.abs(val - rval).max()
    err = np.abs(pol - rpol) - (t["prel"] * rpol + t["pabs"])
    assert np.all(err <= 0), (np.abs(pol - rpol) / (rpol + 1e-12)).max()
    if dtype == "bf16":
        assert np.max(0.5 * np.abs(pol - rpol).sum(1)) <= 2e-2


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_net_matches_torch_golden(require_gpu, dtype):
    g = golden()
    net = A.AlphaZero(int(g["blocks"]), int(g["filters"]), weights=g["weights"], dtype=dtype)
    pol, val = net.forward(g["planes"])
    check(pol, val, g["policy"].astype(np.float64), g["value"].astype(np.float64), dtype)


def random_planes(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        gs = A.GameState()
        for _ in range(int(rng.integers(0, 60))):
            idx = gs.position.legal_indices()
            if len(idx) == 0 or int(A.play_move(gs, int(rng.choice(idx)))) != 0:
                break
        if len(gs.position.legal_indices()):
            out.append(A.to_tensor(gs.position)[0])
    return np.stack(out)


@pytest.mark.parametrize("blocks,filters,dtype,n", [(6, 64, "f32", 24), (6, 64, "bf16", 24), (2, 128, "bf16", 9),
                                                    (2, 128, "f32", 9), (2, 32, "f32", 17),
                                                    (20, 256, "bf16", 6), (20, 256, "f32", 6)])
def test_net_matches_oracle(require_gpu, blocks, filters, dtype, n):
    w = A.random_weights(blocks, filters, seed=42)
    planes = random_planes(n, blocks * 1000 + filters)
    net = A.AlphaZero(blocks, filters, weights=w, dtype=dtype)
    pol, val = net.forward(planes)
    ref = O.RefNet(blocks, filters, w)
    rpol, rval = ref.forward(planes, threads=16)
    check(pol, val, rpol.astype(np.float64), rval.astype(np.float64), dtype)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_rows_are_batch_independent(require_gpu, dtype):
    """Every row is computed independently of the batch it sits in (needed for replay parity
    and for the FEN-cache equivalence, tree.rs:214)."""
    planes = random_planes(13, 5)
    net = A.AlphaZero(2, 64, dtype=dtype)
    pol, val = net.forward(planes)
    for i in (0, 5, 12):
        p1, v1 = net.forward(planes[i:i + 1])
        assert np.array_equal(p1[0], pol[i]) and v1[0] == val[i]
    p2, v2 = net.forward(np.concatenate([planes[7:], planes[:7]]))
    assert np.array_equal(p2[:6], pol[7:]) and np.array_equal(v2[6:], val[:7])


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("blocks,filters", [(2, 32), (6, 64), (2, 128), (20, 256)])
def test_fused_tower_matches_per_layer_kernels(require_gpu, blocks, filters, dtype, monkeypatch):
    """tower_kernel / tower32_kernel (whole tower + heads in one launch, activations resident
    in LDS) against the per-layer conv3x3_kernel + heads_kernel path on the same weights."""
    w = A.random_weights(blocks, filters, seed=7)
    planes = random_planes(37, 11)
    monkeypatch.setenv("AZ_FUSED_TOWER", "1")
    fused = A.AlphaZero(blocks, filters, weights=w, dtype=dtype)
    pf, vf = fused.forward(planes)
    monkeypatch.setenv("AZ_FUSED_TOWER", "0")
    layered = A.AlphaZero(blocks, filters, weights=w, dtype=dtype)
    pl, vl = layered.forward(planes)
    if dtype == "bf16":
        # same bf16 arithmetic, but the fused path adds the bias before the K sum (accumulator
        # init): occasional bf16 rounding flips -> bf16-scale tolerance
        np.testing.assert_allclose(vf, vl, atol=2e-3)
        np.testing.assert_allclose(pf, pl, rtol=2e-2, atol=1e-6)
    else:
        # f32: same products, bias added first vs last and MFMA vs VALU heads -> f32 rounding only
        np.testing.assert_allclose(vf, vl, atol=1e-5)
        np.testing.assert_allclose(pf, pl, rtol=1e-4, atol=1e-8)


def test_mpk_model_file_drives_the_engine(require_gpu, tmp_path):
    """model.save_file -> load_model (training.rs:269-270, main.rs:109-116) -> identical outputs."""
    w = A.random_weights(2, 32, seed=12)
    net = A.AlphaZero(2, 32, weights=w, dtype="f32")
    p = tmp_path / "iteration_3_elo_0.mpk"
    net.save_file(p)
    back = A.load_model(p, 2, 32, dtype="f32")
    x = np.stack([A.to_tensor(A.Position.startpos())[0]] * 3)
    a, b = net.forward(x), back.forward(x)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("blocks,filters", [(6, 64), (2, 128), (20, 256)])
def test_winograd_tower_matches_direct_tower(require_gpu, blocks, filters, monkeypatch):
    """tower32w_kernel<F> (residual convs as Winograd F(2x2,3x3)) against tower32_kernel<F> (direct
    3x3) on the same f32 weights: f32 rounding only (tolerance as the f32 oracle checks)."""
    w = A.random_weights(blocks, filters, seed=3)
    planes = random_planes(41, 13)
    monkeypatch.setenv("AZ_WINOGRAD", "1")
    wn = A.AlphaZero(blocks, filters, weights=w, dtype="f32")
    assert wn.tower_kernel.startswith("tower32w_kernel<%d>" % filters)
    pw, vw = wn.forward(planes)
    monkeypatch.setenv("AZ_WINOGRAD", "0")
    dn = A.AlphaZero(blocks, filters, weights=w, dtype="f32")
    assert dn.tower_kernel.startswith("tower32_kernel<%d>" % filters)
    pd, vd = dn.forward(planes)
    np.testing.assert_allclose(vw, vd, atol=1e-5)
    np.testing.assert_allclose(pw, pd, rtol=1e-4, atol=1e-8)


def test_headline_net_many_positions_and_search_rows(require_gpu):
    """The headline network (20x256 f32, tower32w_kernel<256>) on 64 random-playout positions
    through AlphaZero::forward, and on the rows the search itself evaluated (search mode: the heads
    write the priors straight into the new nodes' edges) for 48 games x 3 simulations from random
    histories -- every row within the f32 tolerance of the oracle network."""
    B, F = 20, 256
    w = A.random_weights(B, F, seed=42)
    net = A.AlphaZero(B, F, weights=w, dtype="f32")
    ref = O.RefNet(B, F, w)
    planes = random_planes(64, 2026)
    pol, val = net.forward(planes)
    rpol, rval = ref.forward(planes, threads=16)
    check(pol, val, rpol.astype(np.float64), rval.astype(np.float64), "f32")
    # search-mode rows
    rng = np.random.default_rng(9)
    hs = []
    while len(hs) < 48:
        gs, h = A.GameState(), []
        for _ in range(int(rng.integers(0, 80))):
            idx = gs.position.legal_indices()
            a = int(rng.choice(idx))
            if int(A.play_move(gs, a)) != 0:
                break
            h.append(a)
        else:
            if len(gs.position.legal_indices()):
                hs.append(h)
    s = A.BatchedSearch(net, games=len(hs), sims=3, seed=4, record_evals=True, eval_log_cap=1024, cache_capacity=0)
    s.set_roots(hs, apply_noise=False)
    s.run()
    keys, vals, off, idx, pri = s.eval_log()
    # the rows evaluated on the roots and on their children (most leaves of a 3-simulation search;
    # deeper leaves are not looked up)
    pos = {}
    for h in hs:
        p = A.Position.startpos()
        for a in h:
            p = p.play(a)
        pos.setdefault(p.fen_key(), p)
        for i in np.unique(p.legal_indices()):
            q = p.play(int(i))
            pos.setdefault(q.fen_key(), q)
    rows = [r for r in range(len(keys)) if int(keys[r]) in pos]
    assert len(rows) >= 64
    x = np.concatenate([A.to_tensor(pos[int(keys[r])]) for r in rows])
    rp, rv = ref.forward(x, threads=16)
    for k, r in enumerate(rows):
        assert abs(float(vals[r]) - float(rv[k])) <= 1e-5
        ii = idx[off[r]:off[r + 1]]
        assert np.all(np.abs(pri[off[r]:off[r + 1]] - rp[k][ii]) <= 1e-4 * rp[k][ii] + 1e-8)

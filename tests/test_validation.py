"""Arena move-choice rules and Elo (validation.rs / ratings.rs) on CPU."""
import numpy as np
import pytest

import azchess as A
import oracle as O
from azchess import validation as V


def test_compute_elos_fixed_point():
    # two players: Elo difference -> 400*log10(w/(1-w)) (ratings.rs:113-143; player 0 pinned)
    for w in (0.25, 0.5, 0.8):
        e = A.compute_elos([[0.5, 1 - w], [w, 0.5]], 150.0)
        assert e[0] == 150.0
        assert e[1] - 150.0 == pytest.approx(400 * np.log10(w / (1 - w)), abs=0.5)   # 1000 steps of rate 8
    # three players from Bradley-Terry ratings 0 / 100 / -200: recovered
    r = np.array([0.0, 100.0, -200.0])
    wm = [[0.5 if i == j else 1 / (1 + 10 ** ((r[j] - r[i]) / 400)) for j in range(3)] for i in range(3)]
    e = A.compute_elos(wm, 0.0)
    assert np.allclose(e, r, atol=0.5)


def test_argmax_is_the_last_maximum():
    assert V.argmax_last([0.1, 0.3, 0.3, 0.2]) == 2          # Rust max_by keeps the later equal element
    assert V.argmax_last([0.5, 0.0, 0.0]) == 0


def test_weighted_index_semantics():
    w = np.zeros(4096, np.float32)
    w[[10, 20, 4000]] = [0.25, 0.5, 0.25]
    assert V.weighted_index(w, 0.0) == 10
    assert V.weighted_index(w, 0.2499) == 10
    assert V.weighted_index(w, 0.25) == 20                    # first cumulative weight > x
    assert V.weighted_index(w, 0.9999999) == 4000
    rng = np.random.default_rng(0)
    cnt = np.bincount([V.weighted_index(w, rng.random()) for _ in range(4000)], minlength=4096)
    assert set(np.nonzero(cnt)[0]) == {10, 20, 4000}
    assert abs(cnt[20] / 4000 - 0.5) < 0.05


def test_stochastic_threshold_is_strict():
    p = np.zeros(4096, np.float32)
    p[[3, 7]] = [0.9, 0.1]
    # fullmoves > 15 -> argmax; at exactly 15 the move is still sampled (validation.rs:297)
    assert V.choose(p, 16, 15, 0.95) == 3
    assert V.choose(p, 15, 15, 0.95) == 7


def test_compute_elos_matches_oracle():
    """azchess.compute_elos against the oracle's C restatement of ratings.rs:113-144 (f32, powf)."""
    rng = np.random.default_rng(7)
    for n in (2, 3, 5, 8):
        w = rng.uniform(0.05, 0.95, (n, n)).astype(np.float32)
        wm = np.triu(w, 1) + np.tril(1.0 - w.T, -1)
        np.fill_diagonal(wm, 0.5)
        for base in (0.0, 150.0, 1200.0):
            a = np.asarray(A.compute_elos(wm, base), np.float64)
            r = np.asarray(O.compute_elos(wm, base), np.float64)
            assert np.allclose(a, r, rtol=1e-6, atol=1e-6 * abs(base) + 1e-4), (n, base, a, r)


def test_choose_matches_oracle():
    """The arena's move choice (validation.rs:297-308) against ref_arena_choose on random sparse
    policies, both sides of the strict threshold, with ties."""
    rng = np.random.default_rng(11)
    for trial in range(300):
        p = np.zeros(4096, np.float32)
        idx = rng.choice(4096, int(rng.integers(1, 40)), replace=False)
        p[idx] = rng.integers(1, 6, len(idx)).astype(np.float32)   # small integers: ties are common
        p /= p.sum()
        fm = int(rng.integers(10, 20))
        u = np.float32(rng.random(dtype=np.float32))
        assert V.choose(p, fm, 15, u) == O.arena_choose(p, fm, 15, u), trial

"""GPU search (select/expand/backup kernels, noise, move choice) against the oracle's
restatement of tree.rs / training.rs.  Bar: BIT-EXACT visit counts, chosen actions, search
depths and final values -- with the synthetic evaluator (identical definition on both
sides) and with the network's own evaluations replayed into the oracle."""
import numpy as np
import pytest

import azchess as A
import oracle as O

pytestmark = pytest.mark.gpu


def histories(n, seed, max_len=30):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        gs, h = A.GameState(), []
        for _ in range(int(rng.integers(0, max_len))):
            idx = gs.position.legal_indices()
            a = int(rng.choice(idx))
            if int(A.play_move(gs, a)) != 0:
                break
            h.append(a)
        else:
            pass
        if int(gs.position.outcome()) == 0 and len(gs.position.legal_indices()):
            # only roots whose history did not already end the game
            ok = True
            g2 = A.GameState()
            for a in h:
                ok &= int(A.play_move(g2, a)) == 0
            if ok:
                out.append(h)
    return out


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("noise", [False, True])
@pytest.mark.parametrize("sims", [16, 100])
def test_search_synthetic_bit_exact(require_gpu, noise, sims, fused, monkeypatch):
    """fused = 1: k_step (backup + select + expand in one launch); 0: separate k_select /
    k_expand / k_backup launches."""
    monkeypatch.setenv("AZ_FUSED_STEPS", fused)
    hs = histories(12, sims + noise)
    s = A.BatchedSearch(None, games=len(hs), sims=sims, noise=noise, seed=11)
    s.set_roots(hs, apply_noise=noise)
    imp, vis, dep = s.run()
    cfg = O.make_cfg(sims=sims, noise=noise, seed=11, eval_kind=0)
    for g, h in enumerate(hs):
        key = O.lib().ref_stream_key(11, g, len(h), 0)
        rv, ri, rd, _ = O.search_game(cfg, h, noise=noise, noise_key=key)
        assert np.array_equal(vis[g].astype(np.float32), rv), g
        assert np.array_equal(imp[g], ri), g
        assert dep[g] == rd


def compare_steps(gpu_steps, ref_steps):
    gs = sorted(gpu_steps, key=lambda s: (s.game_id, s.ply))
    rs = sorted(ref_steps, key=lambda s: (s["game"], s["ply"]))
    assert len(gs) == len(rs)
    for a, b in zip(gs, rs):
        assert (a.game_id, a.ply, a.action, a.search_depth, a.result) == \
               (b["game"], b["ply"], b["action"], b["depth"], b["result"]), (a.game_id, a.ply)
        assert a.visits == {k: int(v) for k, v in b["visits"].items()}
        assert np.float32(a.final_value) == np.float32(b["final_value"])


def test_selfplay_synthetic_bit_exact(require_gpu):
    games, sims = 6, 16
    avg, steps = A.run_all_episodes(None, games=games, sims=sims, seed=5)
    ref, rsims, _ = O.selfplay(O.make_cfg(sims=sims, noise=True, seed=5, eval_kind=0), games)
    compare_steps(steps, ref)
    assert {s.game_id for s in steps} == set(range(games))


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_selfplay_net_replay_bit_exact(require_gpu, dtype):
    """Self-play with the 2x32 network; the oracle replays the GPU's evaluations and must
    reproduce every visit count / action / depth / final value.  The evaluations
    themselves are checked against the oracle network within the dtype tolerance."""
    games, sims = 4, 16
    w = A.random_weights(2, 32, seed=42)
    net = A.AlphaZero(2, 32, weights=w, dtype=dtype)
    sp = A.SelfPlay(net, games=games, sims=sims, seed=9, record_evals=True, eval_log_cap=1 << 17)
    sp.reset()
    steps = []
    for _ in range(600):
        _, active = sp.step()
        steps += sp.drain()
        if active == 0:
            break
    keys, vals, off, idx, pri = sp.search.eval_log()
    rep = O.Replay(keys, vals, off, idx, pri)
    ref, _, _ = O.selfplay(O.make_cfg(sims=sims, noise=True, seed=9, eval_kind=2), games, replay=rep)
    compare_steps(steps, ref)
    # evaluations vs the oracle network (first 64 logged rows)
    ref_net = O.RefNet(2, 32, w)
    pos_by_key = {}
    for s in steps:
        pos_by_key.setdefault(s.state.fen_key(), s.state)
    tol = {"bf16": (2e-2, 5e-2, 2e-5), "f32": (1e-5, 1e-4, 1e-8)}[dtype]
    checked = 0
    for r in range(len(keys)):
        p = pos_by_key.get(int(keys[r]))
        if p is None:
            continue
        rpol, rval = ref_net.forward(A.to_tensor(p))
        assert abs(vals[r] - rval[0]) <= tol[0]
        ii = idx[off[r]:off[r + 1]]
        assert np.all(np.abs(pri[off[r]:off[r + 1]] - rpol[0][ii]) <= tol[1] * rpol[0][ii] + tol[2])
        checked += 1
        if checked >= 64:
            break
    assert checked > 10


def test_large_batch_invariants(require_gpu):
    """C3-sized batch (2048 games, 20x256 bf16) for a few simulations: size-independent
    properties -- root visit sums equal the simulations run, priors are distributions."""
    net = A.AlphaZero(20, 256, dtype="bf16")
    G, S = 2048, 4
    s = A.BatchedSearch(net, games=G, sims=S, seed=1)
    s.set_roots([[]] * G, apply_noise=True)
    imp, vis, dep = s.run()
    assert np.all(vis.sum(1) == S)
    assert np.allclose(imp.sum(1), 1.0, atol=1e-6)
    st = s.stats()
    assert st["sims"] == G * S and st["evals"] + st["cache_hits"] == st["sims"] - st["terminal_leaves"]


def test_fen_cache_changes_only_the_eval_count(require_gpu):
    """tree.rs:214-219: a cache hit returns exactly what the network would return, so the
    games are identical with the cache on or off; only the number of network rows drops."""
    games, sims = 8, 32
    net = A.AlphaZero(2, 32, dtype="bf16")
    runs = {}
    for cap in (0, 500000):
        sp = A.SelfPlay(net, games=games, sims=sims, seed=21, cache_capacity=cap)
        sp.reset()
        for _ in range(12):
            sp.step()
        st = sp.search.stats()
        runs[cap] = (st, [(s.game_id, s.ply, s.action, tuple(sorted(s.visits.items()))) for s in sp.drain()])
    (st0, s0), (st1, s1) = runs[0], runs[500000]
    assert st0["sims"] == st1["sims"]
    assert st1["cache_hits"] > 0 and st1["evals"] < st0["evals"]
    assert st1["evals"] + st1["cache_hits"] == st0["evals"]


def test_fen_cache_search_bit_exact(require_gpu):
    hs = histories(16, 77)
    s = A.BatchedSearch(None, games=len(hs), sims=200, noise=True, seed=4, cache_capacity=1 << 16)
    s.set_roots(hs, apply_noise=True)
    imp, vis, dep = s.run()
    assert s.stats()["cache_hits"] > 0
    cfg = O.make_cfg(sims=200, noise=True, seed=4, eval_kind=0)
    for g, h in enumerate(hs):
        rv, ri, rd, _ = O.search_game(cfg, h, noise=True, noise_key=O.lib().ref_stream_key(4, g, len(h), 0))
        assert np.array_equal(vis[g].astype(np.float32), rv) and dep[g] == rd


def test_search_survives_nan_network(require_gpu):
    """A diverged network (NaN everywhere) must not take the engine out of bounds: every PUCT
    value is NaN, nothing beats -inf, and the walk takes the first edge (the reference keeps
    its initial index, tree.rs:121-131).  The search completes with every simulation counted."""
    w = A.random_weights(2, 32, seed=5)
    w[:] = np.nan
    net = A.AlphaZero(2, 32, weights=w, dtype="bf16")
    s = A.BatchedSearch(net, games=4, sims=64, seed=1)
    s.set_roots([[], [588], [], [588]], apply_noise=True)
    imp, vis, dep = s.run()
    assert np.all(vis.sum(axis=1) == 64)
    assert np.all((dep >= 1) & (dep <= 64))


@pytest.mark.parametrize("cache", [0, 1 << 16])
def test_fused_step_kernel_matches_separate_kernels(require_gpu, monkeypatch, cache):
    """k_step (backup of step i-1 + select + expand of step i in one launch) against the
    separate k_select / k_expand / k_backup launches, and against the timed mix (every 8th
    step separate): identical games, visit counts, evaluations and cache hits."""
    net = A.AlphaZero(2, 32, dtype="bf16")
    runs = []
    for fused, timing in ((True, False), (False, False), (True, True)):
        monkeypatch.setenv("AZ_FUSED_STEPS", "1" if fused else "0")
        sp = A.SelfPlay(net, games=12, sims=40, seed=13, cache_capacity=cache)
        sp.reset()
        sp.search.timing(reset=True, enable=timing)
        for _ in range(6):
            sp.step()
        st = sp.search.stats()
        runs.append(((st["sims"], st["evals"], st["terminal_leaves"], st["cache_hits"]),
                     sorted((s.game_id, s.ply, s.action, s.search_depth, tuple(sorted(s.visits.items())))
                            for s in sp.drain())))
    assert runs[0][0][0] == 12 * 40 * 6
    assert runs[0] == runs[1] == runs[2]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("timing", [False, True])
def test_persistent_sims_match_step_kernels(require_gpu, monkeypatch, timing, dtype):
    """k_sims32w (each game's simulation loop in one workgroup: backup, select, expand and the
    evaluation -- Winograd f32 or the bf16 tower -- with no grid-wide step boundary) against
    k_step + the batched tower, and
    against the timed mix (every 32nd simulation step through the separate kernels): identical
    visit counts, improved policies and depths of one search, identical simulation / evaluation /
    terminal-leaf counts over several self-play moves."""
    net = A.AlphaZero(6, 64, weights=A.random_weights(6, 64, seed=42), dtype=dtype)
    runs = []
    for persist in ("1", "0"):
        monkeypatch.setenv("AZ_PERSIST", persist)
        s = A.BatchedSearch(net, games=24, sims=300, seed=29, cache_capacity=0)
        s.timing(reset=True, enable=timing)
        s.set_roots([[]] * 12 + [[588]] * 12, apply_noise=True)
        assert s.persistent == (persist == "1")
        imp, vis, dep = s.run()
        st = s.stats()
        sp = A.SelfPlay(net, games=24, sims=72, seed=31, cache_capacity=0)
        sp.reset()
        sp.search.timing(reset=True, enable=timing)
        for _ in range(5):
            sp.step()
        st2 = sp.search.stats()
        runs.append((imp, vis, dep, (st["sims"], st["evals"], st["terminal_leaves"], st["overflow"]),
                     (st2["sims"], st2["evals"], st2["terminal_leaves"], st2["overflow"])))
    (i1, v1, d1, a1, b1), (i0, v0, d0, a0, b0) = runs
    assert a1[0] == 24 * 300 and a1[3] == 0 and b1[0] == 24 * 72 * 5 and b1[3] == 0
    assert np.array_equal(v1, v0) and np.array_equal(i1, i0) and np.array_equal(d1, d0)
    assert a1 == a0 and b1 == b0


def test_selfplay_matches_committed_search_golden(require_gpu):
    """C1 (BASELINE.json configs[0]: 16 simulations per move) on the GPU against the committed
    golden vectors (tests/golden/search_c1.npz, synthetic evaluator, 2 whole games): every
    EpisodeStep's action, depth, result, final value and root visit counts bit-exact."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "search_c1.npz"))
    _, steps = A.run_all_episodes(None, games=2, sims=16, seed=5)
    steps = sorted(steps, key=lambda s: (s.game_id, s.ply))
    assert len(steps) == len(g["synth_ply"])
    off = g["synth_vis_off"]
    for i, s in enumerate(steps):
        assert (s.game_id, s.ply, s.action, s.search_depth, s.result) == \
               tuple(int(g["synth_" + k][i]) for k in ("game", "ply", "action", "depth", "result")), i
        assert np.float32(s.final_value) == g["synth_final_value"][i], i
        ref = {int(k): float(v) for k, v in zip(g["synth_vis_idx"][off[i]:off[i + 1]], g["synth_vis_n"][off[i]:off[i + 1]])}
        assert s.visits == ref, i


M64 = (1 << 64) - 1


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def synthetic_process_batch(states, calls=None):
    """A caller-owned evaluator (process_batch, training.rs:380-422, written outside the engine)
    that restates the synthetic evaluator the oracle shares (net.hip synth_eval_kernel): priors
    1 + splitmix64(key ^ (idx + 1) * phi) >> 48 over the distinct legal indices, normalised in f32;
    value (splitmix64(key ^ c) % 2001 - 1000) / 1000.  Unlisted policy entries get garbage: the
    engine must read the row at the legal indices only."""
    n = len(states)
    if calls is not None:
        calls.append(n)
    pol = np.full((n, 4096), 7.0, np.float32)
    val = np.zeros(n, np.float32)
    for r, p in enumerate(states):
        key = p.fen_key()
        idx = np.unique(p.legal_indices())
        w = [1 + (_splitmix64(key ^ (((int(i) + 1) * 0x9E3779B97F4A7C15) & M64)) >> 48) for i in idx]
        tot = np.float32(sum(w))
        pol[r, idx] = np.array(w, np.float32) / tot
        val[r] = np.float32(int(_splitmix64(key ^ 0x5BD1E9955BD1E995) % 2001) - 1000) / np.float32(1000.0)
    return pol, val


@pytest.mark.parametrize("fused", ["1", "0"])
def test_callback_evaluator_reproduces_synthetic_bit_exact(require_gpu, monkeypatch, fused):
    """AZ_EVAL_CALLBACK (az_search_set_evaluator, the reference's InferenceRequest / process_batch
    boundary): a Python evaluator equal to the synthetic one gives bit-identical visits, improved
    policies and depths -- through the search API and through whole self-play games -- with one
    batched call per simulation step (plus the root evaluation)."""
    monkeypatch.setenv("AZ_FUSED_STEPS", fused)
    hs = histories(6, 41)
    S = 24
    calls = []
    cb = A.BatchedSearch(None, games=len(hs), sims=S, noise=True, seed=17,
                         evaluator=lambda st: synthetic_process_batch(st, calls))
    ref = A.BatchedSearch(None, games=len(hs), sims=S, noise=True, seed=17)
    for s in (cb, ref):
        s.set_roots(hs, apply_noise=True)
    a, b = cb.run(), ref.run()
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert 2 <= len(calls) <= 1 + S and calls[0] == len(hs) and max(calls) <= len(hs)   # no call for an empty step
    st_cb, st_ref = cb.stats(), ref.stats()
    assert (st_cb["sims"], st_cb["evals"], st_cb["terminal_leaves"]) == \
           (st_ref["sims"], st_ref["evals"], st_ref["terminal_leaves"])
    assert sum(calls[1:]) == st_cb["evals"]
    # whole games through the self-play driver (run_all_episodes with a caller evaluator)
    _, steps_cb = A.run_all_episodes(None, games=3, sims=8, seed=5, evaluator=synthetic_process_batch)
    _, steps_ref = A.run_all_episodes(None, games=3, sims=8, seed=5)
    key = lambda s: (s.game_id, s.ply, s.action, s.search_depth, s.result, np.float32(s.final_value),
                     tuple(sorted(s.visits.items())))
    assert sorted(map(key, steps_cb)) == sorted(map(key, steps_ref))


def test_callback_evaluator_errors_surface(require_gpu):
    def bad(states):
        raise RuntimeError("evaluator down")
    s = A.BatchedSearch(None, games=2, sims=4, seed=1, evaluator=bad)
    with pytest.raises(A._lib.AzError, match="evaluator returned"):
        s.set_roots([[], [588]], apply_noise=False)


def _play_moves(sp, moves, k):
    """`moves` self-play moves: through sp.step() (k = None) or run_sims(k) chunks."""
    done = 0
    while done < moves:
        if k is None:
            sp.step()
            done += 1
        else:
            _, active, move_done = sp.run_sims(k)
            assert (active >= 0) == move_done
            done += move_done
    st = sp.search.stats()
    return ((st["sims"], st["evals"], st["terminal_leaves"], st["moves"], st["overflow"]),
            sorted((s.game_id, s.ply, s.action, s.search_depth, s.result, tuple(sorted(s.visits.items())))
                   for s in sp.drain()))


@pytest.mark.parametrize("evaluator", ["net", "synthetic"])
def test_run_sims_chunks_match_whole_moves(require_gpu, monkeypatch, evaluator):
    """az_selfplay_run_sims (the bench's unit: a move cut into K-simulation chunks) against
    az_selfplay_step (whole moves): identical EpisodeSteps and sims / evals / terminal counts for
    K in {1, 7, 100, S}, timing on and off, persistent kernel on and off (6x64 f32 Winograd net),
    with chunk edges that fall on and off the every-32nd timed steps."""
    S, G, moves = 100, 8, 3
    net = A.AlphaZero(6, 64, weights=A.random_weights(6, 64, seed=42), dtype="f32") if evaluator == "net" else None
    # continuous: the games that end restart in their slot, so every move has work in every slot
    mk = lambda: A.SelfPlay(net, games=G, sims=S, seed=37, continuous=True, cache_capacity=0)
    for persist in (("1", "0") if net is not None else ("0",)):
        monkeypatch.setenv("AZ_PERSIST", persist)
        for timing in (False, True):
            sp = mk()
            sp.reset()
            sp.search.timing(reset=True, enable=timing)
            want = _play_moves(sp, moves, None)
            assert want[0][0] == G * S * moves and want[0][4] == 0
            for k in (1, 7, 100, S):
                sp = mk()
                sp.reset()
                sp.search.timing(reset=True, enable=timing)
                assert _play_moves(sp, moves, k) == want, (persist, timing, k)


def test_set_roots_abandons_a_move_in_progress(require_gpu):
    """a chunked move left half done must not leak its simulation cursor into the
    search API on the same handle (new roots start a fresh move)."""
    s = A.BatchedSearch(None, games=2, sims=16, seed=3, continuous=True)
    sp = A.SelfPlay.__new__(A.SelfPlay)
    sp.search, sp.games = s, 2
    sp.reset()
    assert sp.run_sims(5)[2] is False
    s.set_roots([[], [588]], apply_noise=False)
    imp, vis, dep = s.run()
    assert np.all(vis.sum(1) == 16)
    sp.reset()
    fin, act = sp.step()          # a whole move again: the cursor is at 0
    assert act == 2

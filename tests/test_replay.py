"""ReplayBuffer (memory.rs): the native buffer against the Python restatement
(oracle/memory_ref.py) -- entries bit-exact after merges and evictions, sampling distinct and
uniform, save/load round trip and byte-identical bincode layout."""
import numpy as np

import azchess as A
import memory_ref as M
from azchess.memory import ReplayBuffer


def positions(n, seed):
    """Positions from random playouts, with repeats (transpositions of the opening)."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        gs = A.GameState()
        for _ in range(int(rng.integers(0, 12))):
            idx = gs.position.legal_indices()
            if len(idx) == 0 or int(A.play_move(gs, int(rng.choice(idx)))) != 0:
                break
        out.append(gs.position)
    return out


def step(pos, rng):
    idx = np.unique(pos.legal_indices())
    v = rng.integers(1, 30, len(idx)).astype(np.float32)
    pol = np.zeros(4096, np.float32)
    pol[idx] = v / np.float32(v.sum())
    return A.EpisodeStep(pos, pol, float(np.float32(rng.uniform(-1, 1))), 3)


def test_add_merge_evict_matches_restatement():
    rng = np.random.default_rng(0)
    buf, ref = ReplayBuffer(capacity=40), M.ReplayRef(capacity=40)
    for pos in positions(300, 1):
        st = step(pos, rng)
        assert buf.add(st) == ref.add(pos.fen(), st.improved_policy, st.final_value)
    assert len(buf) == len(ref) == 40
    s = buf.sample(1000, seed=5)                    # batch > len: every entry once
    assert len(s) == 40
    got = {x.state.fen(): x for x in s}
    assert set(got) == set(ref.buffer)
    for fen, (pol, val, cnt) in ref.buffer.items():
        assert np.array_equal(got[fen].policy, pol)
        assert np.float32(got[fen].value) == val
    assert max(c for _, _, c in ref.buffer.values()) > 1       # merges happened


def test_sample_planes_match_to_tensor_and_are_uniform():
    rng = np.random.default_rng(2)
    buf = ReplayBuffer(capacity=1000)
    ps = positions(200, 3)
    for p in ps:
        buf.add(step(p, rng))
    n = len(buf)
    planes, pol, val, states = buf.sample_arrays(64, seed=9)
    assert len({s.fen() for s in states}) == 64                # without replacement
    for i in range(64):
        assert np.array_equal(planes[i].reshape(1, 19, 8, 8), A.to_tensor(states[i]))
    counts = np.zeros(n)
    fens = sorted(s.state.fen() for s in buf.sample(n, seed=0))
    where = {f: i for i, f in enumerate(fens)}
    for seed in range(400):
        for s in buf.sample(8, seed=seed):
            counts[where[s.state.fen()]] += 1
    exp = 400 * 8 / n
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < n + 6 * np.sqrt(2 * n), chi2                # ~ chi2(n-1)


def test_episode_step_add_uses_visit_fractions():
    sp_step = A._lib.AzEpisodeStep()
    sp_step.state = A.Position.startpos()._p
    sp_step.final_value = 0.5
    sp_step.nvis = 3
    for i, (ix, n) in enumerate([(588, 5), (1540, 3), (12, 0)]):
        sp_step.vis_idx[i], sp_step.vis_n[i] = ix, n
    buf = ReplayBuffer(capacity=10)
    assert buf.add(sp_step) == 1
    assert buf.add(sp_step) == 0
    s = buf.sample(1)[0]
    assert s.policy[588] == np.float32(5) / np.float32(8) and s.policy[1540] == np.float32(3) / np.float32(8)
    assert s.policy.sum() == np.float32(1.0) and s.value == 0.5


def test_save_load_round_trip_and_bincode_layout(tmp_path):
    rng = np.random.default_rng(4)
    buf, ref = ReplayBuffer(capacity=30), M.ReplayRef(capacity=30)
    for pos in positions(80, 5):
        st = step(pos, rng)
        buf.add(st)
        ref.add(pos.fen(), st.improved_policy, st.final_value)
    path = tmp_path / "replay_buffer"
    buf.save(path)
    raw = path.read_bytes()
    assert raw == M.encode(ref)
    back = ReplayBuffer.load(path, capacity=30)
    assert len(back) == len(buf)
    a = {s.state.fen(): s for s in buf.sample(100)}
    b = {s.state.fen(): s for s in back.sample(100)}
    assert a.keys() == b.keys()
    for k in a:
        assert np.array_equal(a[k].policy, b[k].policy) and a[k].value == b[k].value
    path.write_bytes(raw[:-3])
    try:
        ReplayBuffer.load(path)
        assert False, "truncated file accepted"
    except A._lib.AzError:
        pass

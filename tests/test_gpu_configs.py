"""The BASELINE.json configurations at their own sizes, in search mode (the fused tower writing
priors straight into the tree), against the oracle.

  C2 (configs[1]): 6x64 net, 800 sims/move -- 64 games, one move: bit-exact visit counts and
      depths against the oracle replaying the GPU's logged evaluations (tree.rs:169-207), and the
      logged evaluations against the oracle network within the dtype tolerance.
  C3 (configs[2]): 2048 games x 800 sims x 20x256 f32, one move: the 800-sim arenas (node/edge
      bump allocators, select path, overflow counter) and size-independent properties, plus the
      oracle replay of 8 sampled games.
Tolerances as in test_gpu_net.py (f32: value 1e-5, policy 1e-4 relative; bf16: 2e-2 / 5e-2)."""
import numpy as np
import pytest

import azchess as A
import oracle as O

pytestmark = pytest.mark.gpu

TOL = {"bf16": (2e-2, 5e-2, 2e-5), "f32": (1e-5, 1e-4, 1e-8)}


def positions_near_start(depth):
    """fen_key -> Position for every position within `depth` plies of the start (the shallow
    part of every search tree from the start position)."""
    out = {}
    frontier = [A.Position.startpos()]
    for d in range(depth + 1):
        nxt = []
        for p in frontier:
            out.setdefault(p.fen_key(), p)
            if d < depth:
                nxt += [p.play(int(i)) for i in p.legal_indices()]
        frontier = nxt
    return out


def replay_check(s, G, S, seed, games):
    keys, vals, off, idx, pri = s.eval_log()
    rep = O.Replay(keys, vals, off, idx, pri)
    cfg = O.make_cfg(sims=S, noise=True, seed=seed, eval_kind=2)
    return rep, cfg, (keys, vals, off, idx, pri)


def check_evals(log, w, blocks, filters, dtype, depth, limit):
    keys, vals, off, idx, pri = log
    near = positions_near_start(depth)
    ref = O.RefNet(blocks, filters, w)
    rows = [r for r in range(len(keys)) if int(keys[r]) in near]
    rng = np.random.default_rng(0)
    rows = sorted(set(rng.choice(rows, min(limit, len(rows)), replace=False).tolist()))
    planes = np.stack([A.to_tensor(near[int(keys[r])])[0] for r in rows])
    rpol, rval = ref.forward(planes, threads=16)
    tv, tr, ta = TOL[dtype]
    for j, r in enumerate(rows):
        assert abs(vals[r] - rval[j]) <= tv, (r, vals[r], rval[j])
        ii = idx[off[r]:off[r + 1]]
        assert np.all(np.abs(pri[off[r]:off[r + 1]] - rpol[j][ii]) <= tr * rpol[j][ii] + ta), r
    return len(rows)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_c2_search_mode_replay_bit_exact(require_gpu, dtype):
    G, S, seed = 64, 800, 17
    w = A.random_weights(6, 64, seed=42)
    net = A.AlphaZero(6, 64, weights=w, dtype=dtype)
    assert net.fused_tower
    s = A.BatchedSearch(net, games=G, sims=S, seed=seed, record_evals=True, eval_log_cap=G * (S + 2),
                        cache_capacity=0)
    s.set_roots([[]] * G, apply_noise=True)
    imp, vis, dep = s.run()
    st = s.stats()
    assert st["sims"] == G * S and st["overflow"] == 0
    rep, cfg, log = replay_check(s, G, S, seed, G)
    for g in range(G):
        rv, ri, rd, _ = O.search_game(cfg, [], noise=True, noise_key=O.lib().ref_stream_key(seed, g, 0, 0), replay=rep)
        assert np.array_equal(vis[g].astype(np.float32), rv), g
        assert np.array_equal(imp[g], ri), g
        assert dep[g] == rd, g
    assert check_evals(log, w, 6, 64, dtype, depth=2, limit=96) >= 32


def test_c3_800_sims_one_move(require_gpu):
    G, S, seed = 2048, 800, 23
    w = A.random_weights(20, 256, seed=42)
    net = A.AlphaZero(20, 256, weights=w, dtype="f32")
    s = A.BatchedSearch(net, games=G, sims=S, seed=seed, record_evals=True, eval_log_cap=G * (S + 2),
                        cache_capacity=0)
    s.set_roots([[]] * G, apply_noise=True)
    imp, vis, dep = s.run()
    st = s.stats()
    # arenas: NMAX = S + 2 nodes, EMAX = NMAX * 218 + 224 edges per game; nothing refused
    assert st["overflow"] == 0
    assert st["max_nodes"] <= st["node_cap"] == S + 2 and st["max_edges"] <= st["edge_cap"]
    assert np.all(vis.sum(1) == S)
    assert np.allclose(imp.sum(1), 1.0, atol=1e-5)
    assert np.all((dep >= 1) & (dep <= S + 1))
    assert st["sims"] == G * S and st["evals"] + st["terminal_leaves"] == G * S
    # 8 sampled games replayed through the oracle with the GPU's own evaluations
    rep, cfg, log = replay_check(s, G, S, seed, G)
    for g in np.random.default_rng(3).choice(G, 8, replace=False):
        rv, ri, rd, _ = O.search_game(cfg, [], noise=True, noise_key=O.lib().ref_stream_key(seed, int(g), 0, 0),
                                      replay=rep)
        assert np.array_equal(vis[g].astype(np.float32), rv), g
        assert dep[g] == rd, g
    assert check_evals(log, w, 20, 256, "f32", depth=1, limit=12) >= 8

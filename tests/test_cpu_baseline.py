"""The CPU baseline of bench.py: the oracle's self-play in lockstep with one batched
evaluation per simulation step must reproduce the per-game oracle bit for bit (same evaluator),
and its torch-CPU network (BN folded, oneDNN convolutions) must match the oracle network within
the f32 tolerance.  CPU only."""
import numpy as np

import azchess as A
import oracle as O
from cpu_net import CpuNet


def _key(s):
    return (s["game"], s["ply"], s["action"], s["depth"], s["result"], np.float32(s["final_value"]),
            tuple(sorted(s["visits"].items())))


def test_batched_selfplay_equals_per_game_oracle():
    cfg = O.make_cfg(sims=16, noise=True, seed=5, eval_kind=0, threads=4)
    a, sa, ea = O.selfplay(cfg, 5)
    b, sb, eb = O.selfplay_batched(cfg, 5)
    assert sorted(map(_key, a)) == sorted(map(_key, b))
    assert (sa, ea) == (sb, eb)


def test_batched_selfplay_with_a_batch_evaluator():
    """The evaluator callback path (process_batch): the oracle net behind it gives the same games
    as the oracle net evaluated per row inside the C loop."""
    w = A.random_weights(2, 32, seed=42)
    ref = O.RefNet(2, 32, w)
    cfg = O.make_cfg(sims=8, noise=True, seed=3, eval_kind=1, net=ref, threads=4)
    calls = []

    def ev(planes):
        calls.append(len(planes))
        return ref.forward(planes)

    a, sa, _ = O.selfplay_batched(cfg, 3, max_plies=6)
    b, sb, eb = O.selfplay_batched(cfg, 3, max_plies=6, evaluator=ev)
    assert sorted(map(_key, a)) == sorted(map(_key, b)) and sa == sb
    assert calls[0] == 1 and max(calls) <= 3 and sum(calls) == eb


def test_cpu_net_matches_oracle_net():
    rng = np.random.default_rng(0)
    for B, F in ((2, 32), (3, 64)):
        w = A.random_weights(B, F, seed=7)
        x = []
        for _ in range(6):
            p = A.Position.startpos()
            for _ in range(int(rng.integers(0, 20))):
                idx = p.legal_indices()
                if len(idx) == 0:
                    break
                p = p.play(int(rng.choice(idx)))
            x.append(A.to_tensor(p)[0])
        x = np.stack(x)
        p1, v1 = CpuNet(B, F, w, threads=4).forward(x)
        p2, v2 = O.RefNet(B, F, w).forward(x)
        assert np.all(np.abs(v1 - v2) <= 1e-5)
        assert np.all(np.abs(p1 - p2) <= 1e-4 * p2 + 1e-8)

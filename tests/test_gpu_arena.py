"""Evaluation arena (validation.rs:155-402) on the GPU: the batched MCTS player (one BatchedSearch
for all of a player's games, fresh noiseless tree per move) replayed move by move against the
oracle's search (synthetic evaluator: identical definition on both sides) -- bit-exact move
lists and results; random and base-model players exercise the other branches."""
import numpy as np
import pytest

import azchess as A
import oracle as O
from azchess import validation as V

pytestmark = pytest.mark.gpu


def test_mcts_arena_matches_oracle_replay(require_gpu):
    G, sims, seed = 6, 12, 3
    p1, p2 = V.Player.mcts(None), V.Player.random()
    res, hist, result = V.evaluate(p1, p2, games=G, sims=sims, seed=seed, max_plies=40, record=True)
    cfg = O.make_cfg(sims=sims, noise=False, seed=0, eval_kind=0)
    for g in range(G):
        gs = A.GameState()
        for ply, a in enumerate(hist[g]):
            white = ply % 2 == 0
            mcts_moves = (g % 2 == 0) == white
            if mcts_moves:
                _, imp, _, _ = O.search_game(cfg, hist[g][:ply], noise=False)
                exp = V.choose(imp, gs.position.fullmoves, 15, V.choice_uniform(seed, g, ply))
                assert a == exp, (g, ply)
            r = int(A.play_move(gs, a))
            if r != 0:
                assert ply == len(hist[g]) - 1
                assert result[g] == {1: 0, 2: 1, 3: -1}[r]
    assert 0.0 <= res.winrate <= 1.0
    # validation.rs:264-268: p2 wins = games - p1 wins - draws (unfinished games count for p2 there)
    assert abs(res.p1_winrate + res.p2_winrate + res.drawrate - 1.0) < 1e-9


def test_base_model_vs_random_and_elo_rankings(require_gpu):
    net = A.AlphaZero(2, 32, dtype="f32", seed=4)
    avg, elos, wm = V.compute_elo_rankings([V.Player.random(), V.Player.base(net)], 150.0, games=8,
                                           max_plies=30)
    assert elos[0] == 150.0 and np.isfinite(elos[1])
    assert wm[1][0] + wm[0][1] == pytest.approx(1.0)

"""Evaluation arena (validation.rs:155-402) on the GPU against the oracle's restatement.

The batched MCTS player (one BatchedSearch for all of a player's games, fresh noiseless tree per
move) is replayed move by move through the oracle: its search (synthetic evaluator, identical
definition on both sides) and its move choice (oracle ref_arena_choose = validation.rs:297-308:
strict `>` threshold, last-max argmax, WeightedIndex) -- bit-exact move lists and results.  The
base-model player's moves are replayed through the oracle network + legal mask (validation.rs:
325-346) + the same choice rule; a move is only excused where the two networks' f32 policies
leave the top two legal entries within the f32 tolerance of test_gpu_net.py."""
import numpy as np
import pytest

import azchess as A
import oracle as O
from azchess import validation as V

pytestmark = pytest.mark.gpu


def u_draw(seed, game, ply):
    # the seeded stand-in for thread_rng (an injected input, not part of the rule under test)
    return np.float32(np.random.default_rng([seed, game, ply]).random(dtype=np.float32))


def test_mcts_arena_matches_oracle_replay(require_gpu):
    G, sims, seed = 6, 12, 3
    p1, p2 = V.Player.mcts(None), V.Player.random()
    res, hist, result = V.evaluate(p1, p2, games=G, sims=sims, seed=seed, max_plies=40, record=True)
    cfg = O.make_cfg(sims=sims, noise=False, seed=0, eval_kind=0)
    for g in range(G):
        og = O.Game()
        for ply, a in enumerate(hist[g]):
            white = ply % 2 == 0
            mcts_moves = (g % 2 == 0) == white
            if mcts_moves:
                _, imp, _, _ = O.search_game(cfg, hist[g][:ply], noise=False)
                exp = O.arena_choose(imp, og.position.fullmoves, 15, u_draw(seed, g, ply))
                assert a == exp, (g, ply)
            r = og.play_index(a)
            assert r >= 0, (g, ply)
            if r != 0:
                assert ply == len(hist[g]) - 1
                assert result[g] == {1: 0, 2: 1, 3: -1}[r]
    assert 0.0 <= res.winrate <= 1.0
    # validation.rs:264-268: p2 wins = games - p1 wins - draws (unfinished games count for p2 there)
    assert abs(res.p1_winrate + res.p2_winrate + res.drawrate - 1.0) < 1e-9


def test_base_model_arena_matches_oracle_replay(require_gpu):
    G, seed = 8, 5
    w = A.random_weights(2, 32, seed=4)
    net = A.AlphaZero(2, 32, weights=w, dtype="f32")
    ref = O.RefNet(2, 32, w)
    res, hist, result = V.evaluate(V.Player.base(net), V.Player.random(), games=G, seed=seed, max_plies=40,
                                   record=True)
    checked = excused = 0
    for g in range(G):
        og = O.Game()
        for ply, a in enumerate(hist[g]):
            if (g % 2 == 0) == (ply % 2 == 0):            # the base model is to move
                pos = og.position
                pol, _ = ref.forward(O.to_tensor(pos))
                masked = O.mask_to_legal(pos, pol[0])
                exp = O.arena_choose(masked, pos.fullmoves, 15, u_draw(seed, g, ply))
                if a != exp:
                    legal = np.sort(masked[masked > 0])
                    gap = legal[-1] - legal[-2] if len(legal) > 1 else 1.0
                    assert gap <= 1e-4 * legal[-1] + 1e-8, (g, ply, a, exp)
                    excused += 1
                checked += 1
            assert og.play_index(a) >= 0
    assert checked > 50 and excused <= 1


def test_same_player_on_both_sides(require_gpu):
    """evaluate(p, p): one MCTS player plays both colours of every game (validation.rs:155-282
    with player_1 == player_2); every game's moves replay through the oracle."""
    G, sims, seed = 4, 8, 2
    p = V.Player.mcts(None)
    res, hist, result = V.evaluate(p, p, games=G, sims=sims, seed=seed, max_plies=12, record=True)
    cfg = O.make_cfg(sims=sims, noise=False, seed=0, eval_kind=0)
    for g in range(G):
        og = O.Game()
        for ply, a in enumerate(hist[g]):
            _, imp, _, _ = O.search_game(cfg, hist[g][:ply], noise=False)
            assert a == O.arena_choose(imp, og.position.fullmoves, 15, u_draw(seed, g, ply)), (g, ply)
            assert og.play_index(a) >= 0
    assert res.p1_winrate + res.p2_winrate + res.drawrate == pytest.approx(1.0)


def test_base_model_vs_random_elo_rankings(require_gpu):
    net = A.AlphaZero(2, 32, dtype="f32", seed=4)
    avg, elos, wm = V.compute_elo_rankings([V.Player.random(), V.Player.base(net)], 150.0, games=8,
                                           max_plies=30)
    ref = O.compute_elos(wm, 150.0)
    assert np.allclose(elos, ref, rtol=1e-6, atol=0)
    assert elos[0] == 150.0
    assert wm[1][0] + wm[0][1] == pytest.approx(1.0)

"""The oracle helpers the device rules tests (tests/test_gpu_rules.py) rely on, checked against the
oracle's per-position functions: batched rules answers, packed fields, searches from a given
GameState.  CPU only."""
import numpy as np

import oracle as O


def test_rules_batch_matches_per_position_oracle():
    parents, actions = O.random_playouts(3, 12, 300)
    assert len(actions) > 1000
    ref = O.rules_batch(parents, actions)
    for i in range(0, len(actions), 37):
        c = O.play_unchecked(parents[i], O.index_to_move(int(actions[i]), parents[i]))
        assert O.to_fen(ref["child"][i]) == O.to_fen(c)
        assert list(ref["moves"][i, :ref["nmoves"][i]]) == list(O.legal_indices(c))
        assert ref["outcome"][i] == O.outcome(c) and ref["in_check"][i] == O.in_check(c)
        assert ref["legal_ep"][i] == O.legal_ep(c) and ref["fen_key"][i] == O.fen_key(c)
        assert np.array_equal(ref["planes"][i], O.to_tensor(c))
    bb, meta = O.pack(ref["child"], len(actions))
    assert np.array_equal(bb[5], O.bitboards(ref["child"][5]))
    assert meta[5, 0] == ref["child"][5].turn and meta[5, 3] == ref["child"][5].halfmoves


def test_random_playouts_are_deterministic_and_reach_the_corners():
    p1, a1 = O.random_playouts(7, 40, 400)
    p2, a2 = O.random_playouts(7, 40, 400)
    assert np.array_equal(a1, a2)
    assert max(p.halfmoves for p in p1) >= 60
    assert any(len(set(O.legal_indices(p).tolist())) < len(O.legal_indices(p)) for p in p1)   # promotions
    t = O.take(p1, [4, 2])
    assert O.to_fen(t[0]) == O.to_fen(p1[4]) and O.to_fen(t[1]) == O.to_fen(p1[2])


def test_search_from_start_equals_history_search():
    """ref_search_from(startpos FEN) == ref_search_game from the startpos; a FEN root searches."""
    cfg = O.make_cfg(sims=64, noise=True, seed=3, eval_kind=0)
    h = [588, 588]
    a = O.search_game(cfg, h, noise=True, noise_key=11)
    b = O.search_game(cfg, h, noise=True, noise_key=11, start=O.startpos())
    assert all(np.array_equal(x, y) for x, y in zip(a[:2], b[:2])) and a[2:] == b[2:]
    v, imp, d, _ = O.search_game(cfg, [], noise=True, noise_key=5,
                                 start=O.from_fen("3k4/8/8/8/8/8/8/3KQ3 b - - 98 150"))
    assert v.sum() == 64 and d >= 1


def test_repetition_history_from_start():
    """GameState from a FEN: the start position counts once (chess.rs:20-26 for the startpos)."""
    g = O.lib()
    import ctypes as C
    st = O.RefGame()
    g.ref_game_from.argtypes = [C.POINTER(O.RefGame), C.POINTER(O.RefPos)]
    p = O.from_fen("4k3/8/8/8/8/8/8/R3K2R w - - 0 1")
    g.ref_game_from(C.byref(st), C.byref(p))
    shuffle = [(7, 15), (60, 59), (15, 7), (59, 60)] * 2
    res = []
    for f, t in shuffle:
        res.append(g.ref_play_move(C.byref(st), O.RefMove(f, t, 0, 0)))
    g.ref_game_free(C.byref(st))
    assert res == [0] * 7 + [1]          # the start position's third occurrence draws

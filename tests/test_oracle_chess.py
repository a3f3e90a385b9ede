"""Pins the CPU oracle's chess layer with known answers: canonical perft
counts, fixed move-index table entries and index round trips."""
import numpy as np
import pytest

import oracle as O

PERFT = [
    ("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", [20, 400, 8902, 197281]),
    ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", [48, 2039, 97862]),
    ("8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1", [14, 191, 2812, 43238]),
    ("r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1", [6, 264, 9467]),
    ("rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8", [44, 1486, 62379]),
    ("r4rk1/1pp1qppp/p1np1n2/2b1p1B1/2B1P1b1/P1NP1N2/1PP1QPPP/R4RK1 w - - 0 10", [46, 2079, 89890]),
]


@pytest.mark.parametrize("fen,counts", PERFT)
def test_perft_known_answers(fen, counts):
    p = O.from_fen(fen)
    assert [O.perft(p, d + 1) for d in range(len(counts))] == counts


def test_index_table_entries():
    # White e2e4 = plane 9 (N, 2) = 588; Black e7e5 mirrored = 588; O-O = 1540
    assert O.move_to_index((12, 28, 0, 0), 0) == 9 * 64 + 1 * 8 + 4
    assert O.move_to_index((52, 36, 0, 0), 1) == 588
    assert O.move_to_index((4, 7, 0, 2), 0) == 24 * 64 + 4
    assert O.move_to_index((4, 0, 0, 2), 0) == 53 * 64 + 4
    # knights: b1c3 plane 0 (1,2), b1a3 plane 7 (-1,2)
    assert O.move_to_index((1, 18, 0, 0), 0) == 0 * 64 + 1
    assert O.move_to_index((1, 16, 0, 0), 0) == 7 * 64 + 1


def test_startpos_order_is_shakmaty_order():
    # pawn single pushes a..h, double pushes a..h, then Nb1-a3, Nb1-c3, Ng1-f3, Ng1-h3
    idx = list(O.legal_indices(O.startpos()))
    assert idx == [520 + f for f in range(8)] + [584 + f for f in range(8)] + [449, 1, 454, 6]


def test_index_round_trip_random_games():
    rng = np.random.default_rng(0)
    for game in range(40):
        g = O.Game()
        for ply in range(120):
            p = g.position
            idx = O.legal_indices(p)
            if len(idx) == 0:
                break
            for i in set(idx.tolist()):
                m = O.index_to_move(int(i), p)
                assert m is not None and O.move_to_index(m, p.turn) == i
            r = g.play_index(int(rng.choice(idx)))
            if r != 0:
                break


def test_underpromotions_duplicate_the_queen_index():
    p = O.from_fen("8/P6k/8/8/8/8/8/K7 w - - 0 1")
    idx = list(O.legal_indices(p))
    q = 7 + 1  # plane N dist 1 -> 8
    assert idx.count(q * 64 + 6 * 8 + 0) == 4


def test_insufficient_material_and_outcomes():
    assert O.outcome(O.from_fen("8/8/8/8/8/8/8/K1k5 w - - 0 1")) == 1           # K vs K
    assert O.outcome(O.from_fen("8/8/8/8/8/8/8/KNk5 w - - 0 1")) == 1           # K+N vs K
    assert O.outcome(O.from_fen("8/8/8/8/8/8/8/KBk1b3 w - - 0 1")) in (0, 1)
    assert O.outcome(O.from_fen("7k/5Q2/6K1/8/8/8/8/8 b - - 0 1")) == 1         # stalemate
    assert O.outcome(O.from_fen("7k/6Q1/6K1/8/8/8/8/8 b - - 0 1")) == 2          # mate, white wins


def test_threefold_repetition_is_a_draw():
    g = O.Game()
    seq = []
    # Ng1-f3 Ng8-f6 Nf3-g1 Nf6-g8 twice -> startpos occurs a third time
    def idx_of(fr, to, turn):
        return O.move_to_index((fr, to, 0, 0), turn)
    for _ in range(2):
        seq += [idx_of(6, 21, 0), idx_of(62, 45, 1), idx_of(21, 6, 0), idx_of(45, 62, 1)]
    res = [g.play_index(i) for i in seq]
    assert res[:-1] == [0] * 7 and res[-1] == 1


def test_dirichlet_is_a_distribution():
    for n in (2, 5, 20, 218):
        x = O.dirichlet(0.3, n, 1234 + n)
        assert x.shape == (n,) and np.all(x >= 0) and abs(float(x.sum()) - 1.0) < 1e-5
    # mean of component 0 over many keys ~ 1/n
    m = np.mean([O.dirichlet(0.3, 4, k)[0] for k in range(4000)])
    assert abs(m - 0.25) < 0.02

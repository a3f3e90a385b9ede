"""Product rules/codec (libaz host entry points, the same chess.h the GPU runs) against
the oracle on random playouts and edge positions: legal index lists (order and
duplicates), play_move results incl. repetition / 50-move / 200-fullmove, to_tensor,
FEN and the FEN key.  CPU only (no device calls)."""
import numpy as np
import pytest

import azchess as A
from azchess import _lib as L
import oracle as O

EDGE_FENS = [
    "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
    "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
    "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1",
    "rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8",
    "8/8/8/2k5/3Pp3/8/8/4K3 b - d3 0 1",          # ep available
    "8/8/8/8/k2Pp2Q/8/8/3K4 b - d3 0 1",          # ep illegal (horizontal pin)
    "8/8/8/2k5/3Pp3/8/8/4KQ2 b - d3 0 1",         # in check by the pushed pawn: ep takes it (round 6: the
                                                  # earlier queen-check version is an impossible check)
    "4k3/8/8/8/8/8/8/R3K2R w KQ - 0 1",
    "r3k2r/8/8/8/8/8/8/R3K2R b KQkq - 0 1",
    "r3k2r/8/8/8/8/5q2/8/R3K2R w KQkq - 0 1",      # castling through check
    "4k3/1P6/8/8/8/8/6p1/4K3 w - - 0 1",          # promotions both sides
    "3k4/8/8/8/8/8/8/3KQ3 b - - 99 150",
    "7k/6Q1/6K1/8/8/8/8/8 b - - 0 1",             # checkmate
    "7k/5Q2/6K1/8/8/8/8/8 b - - 0 1",             # stalemate
    "R6R/3Q4/1Q4Q1/4Q3/2Q4Q/Q4Q2/pp1Q4/kBNN1KB1 w - - 0 1",   # 218 legal moves: the maximum (MAX_EDGES)
]


def same_position(pa, po):
    assert pa.fen() == O.to_fen(po)
    assert list(pa.legal_indices()) == list(O.legal_indices(po))
    assert np.array_equal(A.to_tensor(pa)[0], O.to_tensor(po))
    assert pa.fen_key() == O.fen_key(po)
    assert np.array_equal(pa.bitboards(), O.bitboards(po))
    assert int(pa.outcome()) == O.outcome(po)


@pytest.mark.parametrize("fen", EDGE_FENS)
def test_edge_positions(fen):
    same_position(A.Position.from_fen(fen), O.from_fen(fen))


def test_random_playouts_match_oracle():
    rng = np.random.default_rng(7)
    for game in range(60):
        ga, go = A.GameState(), O.Game()
        for ply in range(400):
            pa, po = ga.position, go.position
            same_position(pa, po)
            idx = pa.legal_indices()
            if len(idx) == 0:
                break
            a = int(rng.choice(idx))
            assert A.index_to_move(a, pa) == a
            ra = int(A.play_move(ga, a))
            ro = go.play_index(a)
            assert ra == ro, (game, ply, pa.fen(), a)
            if ra != 0:
                break


def test_repetition_draw_matches():
    ga, go = A.GameState(), O.Game()
    seq = []
    for _ in range(2):
        seq += [A.move_to_index(6, 21, 0), A.move_to_index(62, 45, 1), A.move_to_index(21, 6, 0),
                A.move_to_index(45, 62, 1)]
    for i, a in enumerate(seq):
        ra, ro = int(A.play_move(ga, a)), go.play_index(a)
        assert ra == ro == (1 if i == len(seq) - 1 else 0)


def test_illegal_index_rejected():
    p = A.Position.startpos()
    assert A.index_to_move(0, p) is None        # a1 has a rook that cannot jump
    with pytest.raises(A.IllegalMove):
        A.play_move(A.GameState(), 0)


# setups shakmaty's Chess::from_setup refuses: the engine sizes a node's edges for
# 218 legal moves, so a root or probe parent outside them must be refused on the host
BAD_FENS = [
    "QQQQQQQQ/QQQQQQQQ/8/8/8/8/8/K6k w - - 0 1",          # too much material (many queens)
    "k7/8/8/8/8/8/3QQQQQ/2QQQQQK w - - 0 1",              # 10 queens, no pawns: promoted excess
    "4k3/8/8/8/8/8/PPPPPPPP/P3K3 w - - 0 1",             # 9 pawns, one on the back rank
    "4k3/8/8/8/8/8/8/P3K3 w - - 0 1",                    # pawn on the first rank
    "4k3/8/8/8/8/8/4R3/4K3 w - - 0 1",                   # side not to move in check
    "4k3/8/8/8/8/8/8/4K3 w - e6 0 1",                    # ep square without the pushed pawn (refused)
    "4k3/8/8/3P4/8/8/8/4K3 w - e6 0 1",                   # ep square a pawn could take, no pushed pawn
    "8/8/8/8/8/8/8/8 w - - 0 1",                         # no kings
    "k7/8/8/8/8/8/8/KK6 w - - 0 1",                      # two white kings
    "4k3/8/8/8/8/5n2/3b4/r3K3 w - - 0 1",                # triple check
    "4r3/8/8/8/4K3/8/8/k3r3 w - - 0 1",                  # two checkers on one line through the king (rooks e8, e1)
    "7k/6q1/8/8/3K4/8/8/b7 w - - 0 1",                    # ... on one diagonal (bishop a1, queen g7)
    "k6R/8/8/8/4P3/8/8/4K3 b - e3 0 1",                  # check the double push e2-e4 could not have given
    "8/8/8/6k1/3PN3/8/8/2B1K3 b - d3 0 1",                # ep with two checkers (the push uncovered one)
    "8/8/8/1k6/3Pp3/8/8/4KQ2 b - d3 0 1",                 # ep, and a queen check the push did not uncover
]


@pytest.mark.parametrize("fen", BAD_FENS)
def test_invalid_setups_refused(fen):
    with pytest.raises(L.AzError):
        A.Position.from_fen(fen)


def test_ep_without_capturer_is_dropped_not_refused():
    """shakmaty validates the ep square as written (pushed pawn present, its squares empty) and keeps
    only the pseudo-legal one: a valid square no pawn can take is absent from the position.
    Restated from shakmaty 0.29 (EnPassant::from_setup); parity unpinned -- the reference only
    parses FENs of positions it produced itself (memory.rs:90)."""
    assert A.Position.from_fen("4k3/8/8/8/4P3/8/8/4K3 b - e3 0 1").fen() == "4k3/8/8/8/4P3/8/8/4K3 b - - 0 1"


@pytest.mark.parametrize("fen,ep", [
    ("8/8/8/6k1/3P4/8/8/2B1K3 b - d3 0 1", "-"),         # the push d2-d4 uncovered the bishop's check
    ("8/8/8/8/3Pp3/8/8/k3K3 b - d3 0 1", "d3"),           # no check, a pawn can take: kept
    ("8/8/8/2k5/3P4/8/8/4K3 b - d3 0 1", "-"),           # the pushed pawn itself gives check
])
def test_possible_ep_checks_accepted(fen, ep):
    assert A.Position.from_fen(fen).fen().split()[3] == ep


def test_aligned_checker_rule_is_about_one_line():
    # a knight and a rook check from different lines: a legal double check
    assert A.Position.from_fen("4k3/8/8/8/8/5n2/8/4rK2 w - - 0 1") is not None


def test_probe_refuses_bad_parent_before_any_device_call():
    """az_rules_probe validates every parent on the host (its device scratch holds MAX_EDGES
    moves); the refusal comes before hipSetDevice, so this runs without a GPU."""
    from azchess.chess import positions_to_array, rules_probe
    good = positions_to_array([A.Position.from_fen("4k3/8/8/8/8/8/8/4K2R w K - 0 1")])
    bad = good.copy()
    bad["castling"] = 2                    # white O-O-O right with no rook on a1
    with pytest.raises(L.AzError, match="castling"):
        rules_probe(bad, [-1])
    queens = good.copy()
    queens["bb"][0, 4] |= 0x00FFFF0000000000   # 16 extra white queens
    queens["bb"][0, 6] |= 0x00FFFF0000000000
    with pytest.raises(L.AzError, match="material"):
        rules_probe(queens, [-1])

"""The DEVICE rules path against the oracle, bit for bit.

The search kernels decide every leaf's legal moves, outcome and repetition key on the GPU with the
wave-parallel generator (search_dev.h leaf_rules / gen_legal_wave), every root's with the serial
one (chess.h gen_legal, k_root_setup), and the towers see a leaf through plane_value staging.
az_rules_probe runs exactly those device functions on given (parent, move index) items; here they
are compared with the oracle's restatement of chess.rs:36-63 / 73-171 / 191-245 (move list order
and under-promotion duplicates, tree.rs:86-89; outcome(); in-check; legal en passant; FEN key;
to_tensor) on

* the edge positions of tests/test_host_rules.py and all their children,
* every node of perft trees, whose leaf counts must equal the canonical perft answers,
* > 100k positions of uniform random playouts (promotions, en passant, checks, 50-move clocks),

and the repetition key is checked to be a function of shakmaty's Chess equality (board, turn,
castling rights, legal ep square) over all of them.  Then whole searches run from FEN roots on the
edge positions with Dirichlet noise on -- a duplicated promotion index, the horizontal en-passant
pin, castling, a 98-halfmove clock, a 199-fullmove clock, a repetition history, 218 legal moves --
and must match the oracle's search (tree.rs:84-289) bit for bit."""
import numpy as np
import pytest

import azchess as A
import azchess._lib as L
from azchess.chess import rules_probe
import oracle as O
from test_host_rules import EDGE_FENS

pytestmark = pytest.mark.gpu

EXTRA_FENS = [
    "n1n5/PPPk4/8/8/8/8/4Kppp/5N1N b - - 0 1",                 # promotions by capture, both sides
    "r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1",                     # every castling right
    "r3k2r/1P6/8/8/8/8/6p1/R3K2R w KQkq - 0 1",                 # rook captures by promotion drop rights
    "4k3/8/8/8/8/8/8/4KB2 w - - 0 1",                           # K+B vs K: insufficient
    "4k3/8/8/8/8/8/8/4KN2 w - - 0 1",                           # K+N vs K: insufficient
    "4kb2/8/8/8/8/8/8/2B1K3 w - - 0 1",                         # bishops on the same colour
    "4kb2/8/8/8/8/8/8/3BK3 w - - 0 1",                          # bishops on different colours
    "8/8/8/8/8/1k6/8/K1q5 w - - 0 1",                           # white checkmated in the corner (the kings apart: adjacent kings are refused)
    "k7/8/1Q6/8/8/8/8/K7 b - - 0 1",                            # black stalemated
    "8/8/8/3k4/3pP3/8/8/3K4 b - e3 0 1",                        # ep capture that gives no discovered check
    "8/8/8/K2pP2r/8/8/8/7k w - d6 0 1",                         # white ep illegal: horizontal pin
    "8/8/3k4/8/2pP4/8/8/3K2B1 b - d3 0 1",                      # ep with a bishop behind the captured pawn
    "4k3/8/8/8/8/8/8/R3K2R w KQ - 99 120",                      # clock about to reach 100
    "rnbqkbnr/pppp1ppp/8/4p3/4P3/8/PPPP1PPP/RNBQKBNR w KQkq e6 0 2",   # ep square not pseudo-legal
]
ALL_FENS = EDGE_FENS + EXTRA_FENS
CHUNK = 20000


def dev_positions(refpos, n):
    """The product's az_pos records of oracle positions (no product code involved: packed fields)."""
    bb, meta = O.pack(refpos, n)
    out = np.zeros(n, L.POS_DTYPE)
    out["bb"] = bb
    for k, f in enumerate(("turn", "castling", "ep", "halfmoves", "fullmoves")):
        out[f] = meta[:, k]
    return out


def compare(dev, ref, n):
    """Every field of the device answers against the oracle's for n items."""
    bb, meta = O.pack(ref["child"], n)
    ch = dev["child"]
    assert np.array_equal(ch["bb"], bb), "child bitboards"
    for k, f in enumerate(("turn", "castling", "ep", "halfmoves", "fullmoves")):
        bad = np.nonzero(ch[f].astype(np.int64) != meta[:, k])[0]
        assert len(bad) == 0, (f, bad[:5])
    col = np.arange(L.MAX_MOVES)[None, :]
    for key, cnt in (("moves", "nmoves"), ("root_moves", "root_n")):
        assert np.array_equal(dev[cnt], ref["nmoves"]), (cnt, np.nonzero(dev[cnt] != ref["nmoves"])[0][:5])
        same = (dev[key] == ref["moves"]) | (col >= ref["nmoves"][:, None])
        assert same.all(), (key, np.nonzero(~same.all(1))[0][:5])
    assert np.array_equal(dev["outcome"], ref["outcome"]), np.nonzero(dev["outcome"] != ref["outcome"])[0][:5]
    assert np.array_equal(dev["in_check"], ref["in_check"])
    lep = ref["legal_ep"]
    assert np.array_equal(ch["flags"] & 1, (lep >= 0).astype(np.uint8)), "legal-ep flag"
    assert np.array_equal(ch["ep"][lep >= 0], lep[lep >= 0])
    assert np.array_equal(dev["fen_key"], ref["fen_key"]), "fen key"
    assert np.array_equal(dev["planes"], ref["planes"]), "to_tensor planes"


def check_rep_keys(children, legal_ep):
    """rep_key must be a function of shakmaty Chess equality and separate unequal positions."""
    canon = {}
    back = {}
    for i in range(len(children)):
        c = children[i]
        k = (c["bb"].tobytes(), int(c["turn"]), int(c["castling"]), int(legal_ep[i]))
        r = int(c["rep_key"])
        assert canon.setdefault(k, r) == r
        assert back.setdefault(r, k) == k


def probe_and_compare(par_o, actions, collect_keys=None):
    """device vs oracle over all items (chunked); returns (device nmoves, device children, oracle children)"""
    n = len(actions)
    nm, dch, och = [], [], []
    for a in range(0, n, CHUNK):
        b = min(n, a + CHUNK)
        po = O.take(par_o, np.arange(a, b))
        act = np.asarray(actions[a:b], np.int32)
        ref = O.rules_batch(po, act)
        dev = rules_probe(dev_positions(po, b - a), act)
        compare(dev, ref, b - a)
        if collect_keys is not None:
            collect_keys.append((dev["child"].copy(), ref["legal_ep"].copy()))
        nm.append(dev["nmoves"])
        dch.append(dev["moves"])
        och.append(ref["child"])
    return nm, dch, och


def test_device_rules_edge_positions(require_gpu):
    parents, actions = [], []
    for fen in ALL_FENS:
        p = O.from_fen(fen)
        parents.append(p)
        actions.append(-1)
        for a in sorted(set(O.legal_indices(p).tolist())):
            parents.append(p)
            actions.append(a)
    keys = []
    probe_and_compare(O.as_pos_array(parents), actions, keys)
    assert len(actions) > 400
    ch = np.concatenate([k[0] for k in keys])
    check_rep_keys(ch, np.concatenate([k[1] for k in keys]))


# perft by the device's move lists, breadth first: the leaf count is the sum of the last level's
# list lengths (under-promotion duplicates included, as perft counts them).  Index moves cannot
# express an under-promotion, so the interior levels must hold no promotion: these positions and
# depths satisfy that (checked below), and their counts are the canonical perft answers.
PERFT = [
    ("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", 5, 4865609),
    ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", 3, 97862),
    ("8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1", 5, 674624),
    ("r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1", 2, 264),
    ("rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8", 1, 44),
    ("r4rk1/1pp1qppp/p1np1n2/2b1p1B1/2B1P1b1/P1NP1N2/1PP1QPPP/R4RK1 w - - 0 10", 3, 89890),
]


@pytest.mark.parametrize("fen,depth,count", PERFT)
def test_device_perft_known_answers(require_gpu, fen, depth, count):
    """GPU perft: every node of the tree through the device generator (compared with the oracle at
    every node), leaf count = the canonical answer."""
    par_o = O.as_pos_array([O.from_fen(fen)])
    actions = np.array([-1], np.int32)
    col = np.arange(L.MAX_MOVES)[None, :]
    for level in range(depth):
        nm, mv, och = probe_and_compare(par_o, actions)
        nm = np.concatenate(nm)
        if level == depth - 1:                   # this level's list lengths sum to perft(depth)
            assert int(nm.sum()) == count
            return
        mv = np.concatenate(mv)
        valid = col < nm[:, None]
        # interior level: no duplicated index (no promotion) -- the precondition of index perft
        srt = np.sort(np.where(valid, mv, -1 - col), axis=1)
        assert not np.any((srt[:, 1:] == srt[:, :-1]) & (srt[:, 1:] >= 0)), "promotion inside the perft tree"
        rows = np.repeat(np.arange(len(nm)), nm)
        actions = mv[valid].astype(np.int32)
        # the next level's parents are the ORACLE's children (the device's were compared, not reused)
        och_all = O.as_pos_array([p for chunk in och for p in chunk])
        par_o = O.take(och_all, rows)


def test_device_rules_random_playouts(require_gpu):
    """> 100k (parent, index) items from uniform random playouts (games to the end: promotions,
    en passant, checks, long quiet stretches up to the 50-move draw)."""
    parents, actions = O.random_playouts(2024, 340, 400, cap=150000)
    n = len(actions)
    assert n >= 100000
    keys = []
    nm, _, _ = probe_and_compare(O.as_pos_array(parents), actions, keys)
    ch = np.concatenate([k[0] for k in keys])
    lep = np.concatenate([k[1] for k in keys])
    check_rep_keys(ch, lep)
    # the sample reaches the rules' corners
    assert (ch["halfmoves"] >= 99).sum() > 50, "50-move clocks"
    assert (lep >= 0).sum() > 100, "legal en passant"
    assert (np.concatenate(nm) == 0).sum() > 20, "mates / stalemates"


# ---------------------------------------------------------------------------- searches from FENs
SEARCH_ROOTS = [
    ("4k3/1P6/8/8/8/8/6p1/4K3 w - - 0 1", []),                   # duplicated promotion index at the root
    ("8/8/8/8/k2Pp2Q/8/8/3K4 b - d3 0 1", []),                   # ep illegal (horizontal pin)
    ("8/8/8/2k5/3Pp3/8/8/4K3 b - d3 0 1", []),                   # ep legal
    ("r3k2r/8/8/8/8/5q2/8/R3K2R w KQkq - 0 1", []),              # castling through check
    ("r3k2r/8/8/8/8/8/8/R3K2R b KQkq - 0 1", []),                # both castlings for Black
    ("3k4/8/8/8/8/8/8/3KQ3 b - - 98 150", []),                   # 50-move draw two plies down
    ("3k4/8/8/8/8/8/8/3KQ3 b - - 0 199", []),                    # 200-fullmove draw one ply down
    ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", []),
    ("R6R/3Q4/1Q4Q1/4Q3/2Q4Q/Q4Q2/pp1Q4/kBNN1KB1 w - - 0 1", []),   # 218 edges: select's > 64 path
    ("7k/8/6K1/8/8/8/Q7/8 w - - 0 1", []),                       # mate in one (Qa8#)
]


def _valid_histories():
    """(fen, history) roots; the histories are built from legal moves: knights out and back from
    the startpos (the root has occurred twice already) and a rook / king shuffle at a 90-move clock."""
    roots = list(SEARCH_ROOTS)
    for fen, tours in (("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
                        ((6, 21), (62, 45), (21, 6), (45, 62), (6, 21), (62, 45))),
                       ("4k3/8/8/8/8/8/8/R3K2R w - - 90 120", ((7, 15), (60, 59), (15, 7), (59, 60)))):
        q, hist = A.Position.from_fen(fen), []
        for f, t in tours:
            a = A.move_to_index(f, t, q.turn)
            q = q.play(a)                        # raises if the move is not legal
            hist.append(a)
        roots.append((fen, hist))
    return roots


@pytest.mark.parametrize("sims,noise", [(64, True), (200, True), (200, False)])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_search_from_fen_roots_bit_exact(require_gpu, monkeypatch, sims, noise, fused):
    """MCTree::new(policy, state, noise) from arbitrary GameStates (tree.rs:84-104) on the edge
    positions, synthetic evaluator: visits, improved policy and depth bit-exact vs the oracle."""
    monkeypatch.setenv("AZ_FUSED_STEPS", fused)
    roots = _valid_histories()
    s = A.BatchedSearch(None, games=len(roots), sims=sims, noise=noise, seed=23, cache_capacity=0)
    s.set_roots([h for _, h in roots], apply_noise=noise, start=[A.Position.from_fen(f) for f, _ in roots])
    imp, vis, dep = s.run()
    cfg = O.make_cfg(sims=sims, noise=noise, seed=23, eval_kind=0)
    for g, (fen, h) in enumerate(roots):
        key = O.lib().ref_stream_key(23, g, len(h), 0)
        rv, ri, rd, _ = O.search_game(cfg, h, noise=noise, noise_key=key, start=O.from_fen(fen))
        assert np.array_equal(vis[g].astype(np.float32), rv), (fen, h)
        assert np.array_equal(imp[g], ri), fen
        assert dep[g] == rd, fen
    st = s.stats()
    assert st["terminal_leaves"] > 0 and st["overflow"] == 0


def test_search_from_fen_roots_persistent_net_replay(require_gpu, monkeypatch):
    """The same roots through the persistent per-game kernel (k_sims32w: expand_leaf_wave<1> beside
    the 6x64 f32 Winograd tower), noise on; the oracle replays the GPU's evaluations and must
    reproduce every root's visits and depth."""
    monkeypatch.setenv("AZ_PERSIST", "1")
    roots = _valid_histories()
    w = A.random_weights(6, 64, seed=42)
    net = A.AlphaZero(6, 64, weights=w, dtype="f32")
    s = A.BatchedSearch(net, games=len(roots), sims=200, noise=True, seed=7, cache_capacity=0, record_evals=True,
                        eval_log_cap=1 << 15)
    assert s.persistent
    s.set_roots([h for _, h in roots], apply_noise=True, start=[A.Position.from_fen(f) for f, _ in roots])
    imp, vis, dep = s.run()
    rep = O.Replay(*s.eval_log())
    cfg = O.make_cfg(sims=200, noise=True, seed=7, eval_kind=2)
    for g, (fen, h) in enumerate(roots):
        rv, _, rd, _ = O.search_game(cfg, h, noise=True, noise_key=O.lib().ref_stream_key(7, g, len(h), 0),
                                     replay=rep, start=O.from_fen(fen))
        assert np.array_equal(vis[g].astype(np.float32), rv) and dep[g] == rd, fen


def test_promotion_root_noise_uses_four_samples(require_gpu):
    """tree.rs:272-289 on a root whose `moves` holds a queen-promotion index 4 times: the Dirichlet
    draws len(moves) samples and that index receives 4 of them, in order -- while the device root
    stores one edge per distinct index.  Bit-exact against the oracle's dense restatement, and the
    promotion edge is searched."""
    fen = "4k3/1P6/8/8/8/8/6p1/4K3 w - - 0 1"
    p = A.Position.from_fen(fen)
    moves = p.legal_indices().tolist()
    promo = [i for i in set(moves) if moves.count(i) == 4]
    assert promo
    s = A.BatchedSearch(None, games=1, sims=400, noise=True, seed=99, cache_capacity=0)
    s.set_roots([[]], apply_noise=True, start=[p])
    imp, vis, dep = s.run()
    cfg = O.make_cfg(sims=400, noise=True, seed=99, eval_kind=0)
    rv, ri, rd, _ = O.search_game(cfg, [], noise=True, noise_key=O.lib().ref_stream_key(99, 0, 0, 0),
                                  start=O.from_fen(fen))
    assert np.array_equal(vis[0].astype(np.float32), rv) and np.array_equal(imp[0], ri) and dep[0] == rd
    assert vis[0][promo[0]] > 0

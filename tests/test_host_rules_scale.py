"""The host rules entry points (chess.h on the CPU: az_pos_play_index / legal_indices / outcome /
encode / fen_key) against the oracle over whole perft trees and >100k random-playout positions --
the same comparisons tests/test_gpu_rules.py makes for the device path, run here through a host
stand-in for az_rules_probe (which needs a GPU).  CPU only."""
import numpy as np
import pytest

import azchess as A
import azchess._lib as L
from azchess.chess import Position
import test_gpu_rules as G


def host_probe(parents, actions, device=0):
    n = len(parents)
    child = np.zeros(n, L.POS_DTYPE)
    mv = np.zeros((n, L.MAX_MOVES), np.int32)
    nm = np.zeros(n, np.int32)
    oc = np.zeros(n, np.int32)
    fk = np.zeros(n, np.uint64)
    planes = np.zeros((n, 19, 8, 8), np.float32)
    for i in range(n):
        pos = Position(L.AzPos.from_buffer_copy(parents[i:i + 1].tobytes()))
        # a played child is finalized by az_pos_play_index; the parent itself through a FEN round trip
        pos = pos.play(int(actions[i])) if actions[i] >= 0 else Position.from_fen(pos.fen())
        child[i:i + 1] = np.frombuffer(bytes(pos._p), L.POS_DTYPE)
        li = pos.legal_indices()
        nm[i] = len(li)
        mv[i, :len(li)] = li
        oc[i] = int(pos.outcome())
        fk[i] = pos.fen_key()
        planes[i] = A.to_tensor(pos)[0]
    return dict(child=child, moves=mv, nmoves=nm, root_moves=mv, root_n=nm, outcome=oc, in_check=None,
                fen_key=fk, planes=planes)


@pytest.fixture
def host_rules(monkeypatch):
    monkeypatch.setattr(G, "rules_probe", host_probe)
    orig = G.compare

    def compare(dev, ref, n):
        dev["in_check"] = ref["in_check"]      # the host ABI does not expose in-check
        orig(dev, ref, n)
    monkeypatch.setattr(G, "compare", compare)


def test_host_rules_edge_positions(host_rules):
    G.test_device_rules_edge_positions(True)


@pytest.mark.parametrize("fen,depth,count", [p for p in G.PERFT if p[2] < 300000])
def test_host_perft_known_answers(host_rules, fen, depth, count):
    G.test_device_perft_known_answers(True, fen, depth, count)


def test_host_rules_random_playouts(host_rules):
    G.test_device_rules_random_playouts(True)

"""The C-ABI library loads on CPU and exports every entry point include/az.h declares."""
import ctypes
import os
import re

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "az.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(az_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ["az_net_create", "az_net_forward", "az_search_create", "az_search_run", "az_search_advance",
              "az_selfplay_step", "az_pos_legal_indices", "az_game_play"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(ROOT, "alphazero-chess_amd", "azchess", "libaz.so"))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    import azchess._lib as L
    bound = {n for n, _, _ in L.SIGNATURES}
    assert set(declared_symbols()) <= bound


def test_struct_sizes():
    import azchess._lib as L
    assert ctypes.sizeof(L.AzPos) == 80
    assert ctypes.sizeof(L.AzSearchStats) == 13 * 8
    assert ctypes.sizeof(L.AzEpisodeStep) == 32 + 80 + 2 * 224 * 2  # az_pos 8-byte aligned

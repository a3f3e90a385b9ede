"""The oracle's self-play (run_episode / MCTree restatement) against the committed C1 search golden
vectors (tests/golden/search_c1.npz, made by tests/golden/make_search_golden.py): every step's
action, depth, result, final value and root visit counts bit-exact, for the synthetic evaluator
and for the 2x32 network.  Pins the oracle against drift (pin 4)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_search_golden as M  # noqa: E402

GOLD = np.load(os.path.join(ROOT, "tests", "golden", "search_c1.npz"))


@pytest.mark.parametrize("name", ["synth", "net"])
def test_oracle_selfplay_matches_search_golden(name):
    got = M.run(name, M.net_weights() if name == "net" else None)
    assert set(got) == {k for k in GOLD.files if k.startswith(name + "_")}
    for k, a in got.items():
        assert a.dtype == GOLD[k].dtype and np.array_equal(a, GOLD[k]), k
    # whole games: every game ends with a result; visits at every step sum to the simulations
    n = np.diff(GOLD[name + "_vis_off"])
    sums = np.add.reduceat(GOLD[name + "_vis_n"], GOLD[name + "_vis_off"][:-1]) if n.all() else None
    assert sums is not None and np.all(sums == M.VARIANTS[name]["sims"])

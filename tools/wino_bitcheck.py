"""Bitwise comparison of two libaz.so builds on the f32 Winograd tower (net.forward) and on one
self-play move (visits / improved policy), e.g. the point-quarter F = 64 conv (AZ_WINO64_PQ=1)
against the one-point-set kernel (AZ_WINO64_PQ=0).  Run once per library with AZ_LIB set:
  AZ_LIB=build_var/x/libaz.so python tools/wino_bitcheck.py dump out_x.npz
then: python tools/wino_bitcheck.py cmp out_a.npz out_b.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "alphazero-chess_amd"))


def dump(path, blocks=6, filters=64):
    import azchess as A
    rng = np.random.default_rng(13)
    planes = (rng.random((97, 19, 8, 8)) < 0.2).astype(np.float32)
    net = A.AlphaZero(blocks, filters, weights=A.random_weights(blocks, filters, seed=3), dtype="f32")
    assert net.tower_kernel.startswith("tower32w_kernel<%d>" % filters), net.tower_kernel
    p, v = net.forward(planes)
    sp = A.SelfPlay(net, games=64, sims=64, seed=5, cache_capacity=0)
    sp.reset()
    sp.step()
    st = sp.search.stats()
    np.savez(path, pol=p, val=v, sims=st["sims"], evals=st["evals"], kernel=net.tower_kernel)
    print("dumped", path, net.tower_kernel, "sims", st["sims"], "evals", st["evals"])


def cmp(a, b):
    A_, B_ = np.load(a), np.load(b)
    ok = True
    for k in ("pol", "val", "sims", "evals"):
        same = np.array_equal(A_[k].view(np.uint32) if A_[k].dtype == np.float32 else A_[k],
                              B_[k].view(np.uint32) if B_[k].dtype == np.float32 else B_[k])
        print("%-6s %s" % (k, "bit-identical" if same else "DIFFERENT (max |d| %g)" % np.abs(A_[k] - B_[k]).max()))
        ok &= same
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])

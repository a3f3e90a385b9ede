"""Per-tensor gradient error of the GPU training step vs the float64 oracle, next to the error of a
float32 torch run of the same oracle (the scale of f32 rounding for this batch)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "alphazero-chess_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import azchess as A  # noqa: E402
import torch  # noqa: E402
import train_ref as T  # noqa: E402
from test_gpu_train import batch  # noqa: E402

for blocks, filters, n in [(2, 32, 16), (6, 64, 8), (20, 256, 2)]:
    w = A.random_weights(blocks, filters, seed=7)
    planes, tpol, tval = batch(n, seed=blocks * 100 + n)
    tr = A.Trainer(blocks, filters, weights=w, max_batch=max(n, 4))
    pl, vl = tr.compute_gradients(planes, tpol, tval)
    g = tr.grads()
    rg, (rpl, rvl) = T.TrainRef(blocks, filters, w).grads(planes, tpol, tval)
    fg, _ = T.TrainRef(blocks, filters, w, dtype=torch.float32).grads(planes, tpol, tval)
    print("== %dx%d B=%d loss gpu %.7f %.7f ref %.7f %.7f" % (blocks, filters, n, pl, vl, rpl, rvl))
    seg, _ = T.segments(blocks, filters)
    for name, (o, shape, bn) in seg.items():
        size = int(np.prod(shape))
        parts = [(name + ".gamma", o, shape[1]), (name + ".beta", o + shape[1], shape[1])] if bn else [(name, o, size)]
        for pname, off, cnt in parts:
            a, r, f = g[off:off + cnt].astype(np.float64), rg[off:off + cnt], fg[off:off + cnt]
            nr = max(np.linalg.norm(r), 1e-30)
            print("%-34s |ref| %.3e  gpu %.2e  torch32 %.2e" % (pname, nr, np.linalg.norm(a - r) / nr,
                                                               np.linalg.norm(f - r) / nr))

"""Profiling driver: the 20x256 tower on 2048 rows, `--iters` forwards (used under
rocprofv3 --pmc to price one conv launch; see profiles/README.md)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-chess_amd"))
import numpy as np  # noqa: E402

import azchess as A  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2048)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--blocks", type=int, default=20)
ap.add_argument("--filters", type=int, default=256)
ap.add_argument("--dtype", default="bf16")
a = ap.parse_args()
net = A.AlphaZero(a.blocks, a.filters, dtype=a.dtype)
rng = np.random.default_rng(0)
planes = (rng.random((a.rows, 19, 8, 8)) < 0.1).astype(np.float32)
for _ in range(a.iters):
    pol, val = net.forward(planes)
print("ok", float(val.mean()))

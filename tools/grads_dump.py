"""Gradients of one 20x256 training step (compute_gradients) on a fixed batch, saved to a .npy:
run once per library build (AZ_LIB) and compare the files bit for bit (kernel-variant checks).
Usage: [AZ_LIB=...] python tools/grads_dump.py out.npy [batch]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "alphazero-chess_amd"))
import numpy as np
import azchess as A

B = int(sys.argv[2]) if len(sys.argv) > 2 else 80
rng = np.random.default_rng(3)
planes = (rng.random((B, 19, 64)) < 0.1).astype(np.float32)
pol = rng.random((B, 4096)).astype(np.float32)
pol /= pol.sum(1, keepdims=True)
val = rng.uniform(-1, 1, B).astype(np.float32)
tr = A.Trainer(20, 256, max_batch=B, seed=42)
pl, vl = tr.compute_gradients(planes, pol, val)
np.save(sys.argv[1], np.concatenate([tr.grads(), np.array([pl, vl], np.float32)]))
print("saved", sys.argv[1], pl, vl)

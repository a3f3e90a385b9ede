"""A few training steps (training.rs:147-190) at 20x256, batch 512, for rocprofv3 kernel stats.
Usage: python tools/train_prof.py [steps] [batch]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "alphazero-chess_amd"))
import numpy as np
import azchess as A

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
rng = np.random.default_rng(1)
planes = (rng.random((B, 19, 64)) < 0.1).astype(np.float32)
pol = rng.random((B, 4096)).astype(np.float32)
pol /= pol.sum(1, keepdims=True)
val = rng.uniform(-1, 1, B).astype(np.float32)
tr = A.Trainer(20, 256, max_batch=B, seed=42)
for i in range(2):
    tr.step(planes, pol, val, A.get_cyclical_lr(i))
t0 = time.perf_counter()
for i in range(steps):
    tr.step(planes, pol, val, A.get_cyclical_lr(i))
print("ms/step", (time.perf_counter() - t0) / steps * 1e3)

"""Summarise an AZ_WINO_TRACE dump (tower32w_kernel, residual block 10 conv1; s_memtime shader
cycles per wave): prologue (chunk 0 transform + barrier), per chunk the MFMA phase and the barrier
wait, the epilogue (output transform + stores) and its barrier.
Usage: python tools/wino_trace.py tower_trace.bin"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], np.uint64).astype(np.int64).reshape(-1, 256)[:, :8 * 24].reshape(-1, 8, 24)[:, :, :24]
t = t[(t[:, :, 0] > 0).all(1) & (t[:, :, 19] > t[:, :, 0]).all(1)]
print("workgroups", len(t))
d = lambda a, b: (t[:, :, b] - t[:, :, a]).ravel()
rows = [("prologue", 0, 1)] + [(f"chunk{c} mfma", 1 + 2 * c if c == 0 else 3 + 2 * (c - 1), 2 + 2 * c) for c in range(8)] + \
       [(f"chunk{c} barrier", 2 + 2 * c, 3 + 2 * c) for c in range(8)] + [("epilogue", 17, 18), ("final barrier", 18, 19),
                                                                          ("layer", 0, 19)]
rows += [("c3 steps 0-7", 7, 20), ("c3 steps 8-15", 20, 21), ("c3 steps 16-23", 21, 22), ("c3 steps 24-31", 22, 23)]
for n, a, b in rows:
    x = d(a, b)
    print("%-16s mean %8.0f  p10 %8.0f  p90 %8.0f" % (n, x.mean(), np.percentile(x, 10), np.percentile(x, 90)))
# per SIMD pair (waves w, w + 4): who finishes chunk 3 first, and by how much
older = t[:, :4, 8] - t[:, :4, 7]
younger = t[:, 4:, 8] - t[:, 4:, 7]
print("chunk3 mfma phase: waves 0-3 mean %.0f, waves 4-7 mean %.0f" % (older.mean(), younger.mean()))
for q in range(4):
    a, b = 20 + q, 20 + q
    x0 = (t[:, :4, a] - t[:, :4, 7]).mean(); x1 = (t[:, 4:, a] - t[:, 4:, 7]).mean()
    print("  after step %2d: waves 0-3 %.0f, waves 4-7 %.0f" % (8 * q + 7, x0, x1))

"""Per-phase cycles of one Winograd conv (AZ_WINO_TRACE, trw stamps of conv1 of the traced block) for
a tower with NCHUNK transform chunks: prologue, per chunk MFMA phase + barrier, epilogue, final barrier.
Usage: python tools/wino_conv64.py tower_trace.bin nwaves nchunk"""
import sys

import numpy as np

NW, NC = int(sys.argv[2]), int(sys.argv[3])
t = np.fromfile(sys.argv[1], np.uint64).astype(np.int64).reshape(-1, 256)[:, :NW * 24].reshape(-1, NW, 24)
t = t[(t[:, :, 0] > 0).all(1) & (t[:, :, 19] > t[:, :, 0]).all(1)]
print("workgroups", len(t))
rows = [("prologue", 0, 1)]
for c in range(NC):
    rows += [("chunk%d mfma" % c, 1 if c == 0 else 1 + 2 * c, 2 + 2 * c), ("chunk%d barrier" % c, 2 + 2 * c, 3 + 2 * c)]
rows += [("epilogue", 1 + 2 * NC, 18), ("final barrier", 18, 19), ("conv", 0, 19)]
for n, a, b in rows:
    x = (t[:, :, b] - t[:, :, a])
    print("%-16s mean %7.0f  p10 %7.0f  p90 %7.0f   per wave %s" % (n, x.mean(), np.percentile(x, 10), np.percentile(x, 90),
                                                               " ".join("%6.0f" % v for v in x.mean(0))))

"""Summarise the coarse per-wave stamps of an AZ_WINO_TRACE dump of tower32w_kernel<F> with <= 4
waves (slots 192 + 16 w + k: 0 start, 1 planes staged, 2 input conv done, 3 + b residual block b
done, 15 heads done); s_memtime shader cycles.
Usage: python tools/wino_coarse.py tower_trace.bin blocks"""
import sys

import numpy as np

B = int(sys.argv[2])
t = np.fromfile(sys.argv[1], np.uint64).astype(np.int64).reshape(-1, 256)[:, 192:256].reshape(-1, 4, 16)
t = t[(t[:, :, 0] > 0).all(1) & (t[:, :, 15] > t[:, :, 0]).all(1)]
extra = t[:, 1, 9:11]   # wave 1's slots 9-10: heads stamps 16-17 of wave 0
print("workgroups", len(t))
seg = [("stage", 0, 1), ("input conv", 1, 2)] + [("block %d" % b, 2 + b, 3 + b) for b in range(B)] + \
      [("heads", 2 + B, 15), ("total", 0, 15)]
if B <= 6:   # heads phases (wave 0's slots 9-11)
    seg += [("heads entry", 2 + B, 12), ("heads prefetch", 12, 13), ("heads A mfma", 13, 14), ("heads A st+bar", 14, 9),
            ("heads A", 2 + B, 9), ("heads B", 9, 25), ("heads C", 25, 26), ("heads sm+bar", 26, 10), ("heads B+C", 9, 10), ("heads slots", 10, 11), ("heads out", 11, 15)]
for n, a, b in seg:
    col = lambda k: extra[:, k - 25:k - 24] if k >= 25 else (t[:, :1, k] if 9 <= k <= 14 else t[:, :, k])
    x = col(b) - col(a) if (a >= 9 or b >= 9) else t[:, :, b] - t[:, :, a]
    x = x.ravel()
    print("%-12s mean %8.0f  p10 %8.0f  p90 %8.0f" % (n, x.mean(), np.percentile(x, 10), np.percentile(x, 90)))

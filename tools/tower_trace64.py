"""Summarise the phase stamps of an AZ_TOWER_TRACE build for a single-chunk Winograd tower (F = 64,
C2; tools/tower_trace.c with 256 games, 6 blocks, 64 filters): cycles per phase of tower32w_board.
Slots as tools/tower_trace.py; per conv only +0 start, +1 chunk transform barrier, +20 step 4,
+12 chunk end, +10 core done, +11 epilogue written.  Usage: python tools/tower_trace64.py trace.bin blocks"""
import sys

import numpy as np

B = int(sys.argv[2]) if len(sys.argv) > 2 else 6
t = np.fromfile(sys.argv[1], np.uint64).astype(np.int64).reshape(8, 8, 2048)[:, :4]   # 4 waves
ok = (t[:, :, 0] > 0).all(1) & (t[:, :, 3 + 64 * 20] > t[:, :, 0]).all(1)
t = t[ok]
print("traced workgroups: %d" % t.shape[0])
conv = np.stack([t[:, :, 3 + 32 * i: 35 + 32 * i] for i in range(2 * B)], 2)
end = 3 + 64 * 20                                    # tower.hip stamps the heads end at a fixed slot
tot = (t[:, :, end] - t[:, :, 0]).mean()
print("total %.0f cycles per board: staging %.0f, input conv %.0f, 2B convs %.0f, heads %.0f"
      % (tot, (t[:, :, 1] - t[:, :, 0]).mean(), (t[:, :, 2] - t[:, :, 1]).mean(),
         (conv[..., -1, 11] - conv[..., 0, 0]).mean(), (t[:, :, end] - conv[:, :, -1, 11]).mean()))
ph = [("residual read + transform + barrier", 0, 1), ("steps 0-4", 1, 20), ("steps 5-end", 20, 12),
      ("(chunk end -> core done)", 12, 10), ("output transform + store", 10, 11)]
for n, a, b in ph:
    print("  %-38s %7.0f" % (n, (conv[..., b] - conv[..., a]).mean()))
print("  between convs (epilogue barrier)       %7.0f" % (conv[..., 1:, 0] - conv[..., :-1, 11]).mean())
print("MFMA per wave per conv: 256 x 32 = 8192 cycles")

h = t[:, :, 1900:1907]
hn = ["weights + 1x1 conv (A)", "barrier", "policy conv + value FC (B, C)", "barrier", "softmax sum + value",
      "barrier"]
print("heads:")
for k in range(6):
    print("  %-38s %7.0f" % (hn[k], (h[..., k + 1] - h[..., k]).mean()))
print("  %-38s %7.0f" % ("priors + value out", (t[:, :, end] - h[..., 6]).mean()))
s0 = t[:, 0, 1910:1916]
if (s0 > 0).all():
    print("simulation (wave 0, last simulation of the traced games):")
    # the kernel's last loop iteration only backs up (no select / expand): its 1912 / 1913 stamps are
    # the previous simulation's, so only intervals within one iteration are printed
    for n, a, b in [("backup", 0, 1), ("expand", 2, 3)]:
        print("  %-38s %7.0f" % (n, (s0[:, b] - s0[:, a]).mean()))

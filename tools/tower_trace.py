"""Summarise the phase stamps of an AZ_TOWER_TRACE build (tools/tower_trace.c): shader-clock cycles
per phase of tower32w_board, mean over the traced workgroups' waves and the 2B residual convs.
Slots per wave: 0 start, 1 planes staged, 2 input conv done, conv i at 3 + 32 i: +0 start, +1 chunk-0
transform barrier, +2+c after chunk c's barrier, +10 core done (before the epilogue), +11 epilogue
written, +12+c before chunk c's barrier, +20+c after step 4 of chunk c; 3 + 64 B: heads done.
Usage: python tools/tower_trace.py trace.bin [blocks]"""
import sys

import numpy as np

B = int(sys.argv[2]) if len(sys.argv) > 2 else 20
NS = 2048
t = np.fromfile(sys.argv[1], np.uint64).astype(np.int64).reshape(8, 8, NS)
wgok = (t[:, :, 0] > 0).all(1)
t = t[wgok]                                           # [wg, waves, NS]
print("traced workgroups: %d" % t.shape[0])
conv = np.stack([t[:, :, 3 + 32 * i: 35 + 32 * i] for i in range(2 * B)], 2)   # [wg, waves, convs, 32]
end = 3 + 64 * 20
total = t[:, :, end] - t[:, :, 0]
print("total %.0f cycles per board; staging %.0f, input conv %.0f, heads %.0f"
      % (total.mean(), (t[:, :, 1] - t[:, :, 0]).mean(), (t[:, :, 2] - t[:, :, 1]).mean(),
         (t[:, :, end] - conv[:, :, -1, 11]).mean()))
per = conv[:, :, :, 11] - conv[:, :, :, 0]
print("conv (start -> epilogue written): mean %.0f  min %.0f  max %.0f" % (per.mean(), per.min(), per.max()))
print("between convs (epilogue barrier + residual reads): mean %.0f" % (conv[:, :, 1:, 0] - conv[:, :, :-1, 11]).mean())
print("xres + chunk-0 transform + barrier: %.0f" % (conv[..., 1] - conv[..., 0]).mean())
print("output transform + resid + relu + store: %.0f" % (conv[..., 11] - conv[..., 10]).mean())
late = np.arange(8) >= 4
for c in range(8):
    start = conv[..., 1 + c]                          # after the barrier that opens chunk c
    s4 = conv[..., 20 + c]
    pre = conv[..., 12 + c]
    post = conv[..., 2 + c]
    print("chunk %d: steps 0-4 %5.0f (early %5.0f late %5.0f)  steps 5-31 %6.0f (early %6.0f late %6.0f)  barrier wait %4.0f (early %4.0f late %4.0f)"
          % (c, (s4 - start).mean(), (s4 - start)[:, ~late].mean(), (s4 - start)[:, late].mean(),
             (pre - s4).mean(), (pre - s4)[:, ~late].mean(), (pre - s4)[:, late].mean(),
             (post - pre).mean(), (post - pre)[:, ~late].mean(), (post - pre)[:, late].mean()))
cyc = (conv[..., 9] - conv[..., 1]).mean() / 8
print("mean chunk (barrier to barrier) %.0f cycles; MFMA work per SIMD per chunk 16384 (2 waves x 256 x 32)" % cyc)
sk = conv.max(1) - conv.min(1)
print("wave skew within a workgroup (max - min), mean: start %.0f, after chunk barriers %.0f, before chunk barriers %.0f, after step 4 %.0f"
      % (sk[..., 0].mean(), sk[..., 2:10].mean(), sk[..., 12:20].mean(), sk[..., 20:28].mean()))

"""Summarise a tower phase trace (AZ_TOWER_TRACE build): per-workgroup s_memrealtime stamps
(100 MHz) at staging end, input conv end, each residual block end and heads end."""
import sys
import numpy as np

TR = 128
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, TR).astype(np.int64)
blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 20
hw = a[:, 47]
a = a[:, :46]
ok = a[:, 0] > 0
a, hw = a[ok], hw[ok]
t0 = a[:, 0].min()
us = lambda x: x / 100.0   # 100 MHz ticks -> us
start = us(a[:, 0] - t0)
end = us(a[:, 45] - t0)
print("workgroups %d  kernel span %.1f us" % (len(a), end.max()))
stage = us(a[:, 1] - a[:, 0])
inconv = us(a[:, 2] - a[:, 1])
blk = us(np.diff(a[:, 2:3 + blocks], axis=1))
heads = us(a[:, 45] - a[:, 2 + blocks])
dur = us(a[:, 45] - a[:, 0])
for name, v in [("stage", stage), ("input conv", inconv), ("block (2 convs)", blk.ravel()), ("heads", heads),
                ("workgroup total", dur)]:
    print("%-16s mean %8.2f  p10 %8.2f  p50 %8.2f  p90 %8.2f  max %8.2f us" % (
        name, v.mean(), np.percentile(v, 10), np.percentile(v, 50), np.percentile(v, 90), v.max()))
print("per-block mean (us):", " ".join("%.1f" % x for x in blk.mean(axis=0)))
# dispatch rounds: sort start times
ss = np.sort(start)
print("start-time quantiles (us):", " ".join("%.0f" % np.percentile(ss, q) for q in (0, 10, 25, 40, 50, 60, 75, 90, 100)))
xcc = (hw >> 32) & 0xF
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
for x in range(8):
    m = xcc == x
    if m.any():
        print("xcc %d: %4d wgs  mean dur %.1f us  last end %.1f us" % (x, m.sum(), dur[m].mean(), end[m].max()))
busy = dur.sum()
print("sum(wg dur) / (span * 256) = %.3f (slot occupancy at 1 wg/CU)" % (busy / (end.max() * 256)))
b = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, TR).astype(np.int64)[ok]
if b.shape[1] >= 114 and (b[:, 112] > 0).all():
    cyc = (b[:, 113] - b[:, 112]).astype(np.float64)
    wall = (b[:, 45] - b[:, 0]) / 100e6
    print("shader clock (s_memtime / wall): mean %.3f GHz  p10 %.3f  p90 %.3f" % (
        (cyc / wall).mean() / 1e9, np.percentile(cyc / wall, 10) / 1e9, np.percentile(cyc / wall, 90) / 1e9))
    w = b[:, 48:112].reshape(-1, 8, 2, 4)          # [wg][wave][conv][start, loop end, epilogue end, barrier end]
    for c in range(2):
        loop = w[:, :, c, 1] - w[:, :, c, 0]
        epi = w[:, :, c, 2] - w[:, :, c, 1]
        bar = w[:, :, c, 3] - w[:, :, c, 2]
        skew = w[:, :, c, 1].max(axis=1) - w[:, :, c, 1].min(axis=1)
        print("block10 conv%d (cycles): loop mean %.0f (min %.0f max %.0f)  epilogue %.0f  barrier wait %.0f  "
              "loop-end skew across waves %.0f" % (c + 1, loop.mean(), loop.min(), loop.max(), epi.mean(), bar.mean(),
                                                  skew.mean()))
    print("ideal MFMA cycles per conv per wave: %d (2 waves/SIMD -> SIMD busy %d)" % (72 * 16 * 16, 2 * 72 * 16 * 16))
    hwid = b[:, 114:122]
    simd = (hwid >> 4) & 3
    for c in range(2):
        end = w[:, :, c, 1] - w[:, :, c, 0].min(axis=1, keepdims=True)
        lo, hi, solo = [], [], []
        for i in range(len(b)):
            for sm in range(4):
                m = simd[i] == sm
                if m.sum() == 2:
                    e = np.sort(end[i][m])
                    lo.append(e[0]); hi.append(e[1])
        lo, hi = np.array(lo), np.array(hi)
        print("conv%d per-SIMD pair: first wave done %.0f, second %.0f cycles after layer start (mean); "
              "SIMD-last spread within WG %.0f" % (c + 1, lo.mean(), hi.mean(),
              np.mean([end[i].max() - np.sort(end[i])[-2] for i in range(len(b))])))
        print("   waves per SIMD histogram:", np.bincount(np.array([(simd[i] == sm).sum() for i in range(len(b)) for sm in range(4)])))
    hh = b[:, 122:125]
    if (hh > 0).all():
        st = b[:, 2 + blocks]
        print("heads phases (us): A %.2f  B+C+max %.2f  sums/value/slots %.2f  outputs %.2f" % (
            ((hh[:, 0] - st) / 100).mean(), ((hh[:, 1] - hh[:, 0]) / 100).mean(), ((hh[:, 2] - hh[:, 1]) / 100).mean(),
            ((b[:, 45] - hh[:, 2]) / 100).mean()))

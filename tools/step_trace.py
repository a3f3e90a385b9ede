"""Summarise the k_step phase stamps of an AZ_STEP_TRACE build (s_memtime = shader-clock cycles,
stamped by lane 0 of each game's wave; the last step recorded in the file).
Usage: python tools/step_trace.py step_trace.bin games"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], np.uint64).astype(np.int64)
G = int(sys.argv[2])
t = t.reshape(-1, G, 16)[-1]
ok = (t[:, 0] > 0) & (t[:, 4] > t[:, 0])
t = t[ok]
names = {(0, 1): "backup", (1, 2): "select", (2, 10): "expand loads", (10, 11): "play_index",
         (11, 8): "attacks+pins", (8, 9): "groups+scans", (9, 5): "edge stores", (5, 6): "repetition+outcome",
         (6, 3): "node/cache", (3, 4): "row alloc", (0, 4): "total"}
for (a, b), n in names.items():
    d = t[:, b] - t[:, a]
    d = d[(t[:, a] > 0) & (t[:, b] > 0)]
    if len(d):
        print("%-20s mean %8.1f  p50 %8.1f  p90 %8.1f  (cycles, %d waves)" % (n, d.mean(), np.median(d), np.percentile(d, 90), len(d)))
span = t[:, 4].max() - t[:, 0].min()
print("launch span %d cycles" % span)

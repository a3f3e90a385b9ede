"""Summarise an AZ_SIMS_TRACE dump (k_sims32w): per game, shader cycles spent in the tree phase
(backup + select + expand on wave 0, the other waves at the barrier) and in the tower phase
(Winograd evaluation of the leaf), accumulated over the persistent launches so far; the last
record in the file is used.  Usage: python tools/sims_trace.py sims_trace.bin games"""
import sys

import numpy as np

G = int(sys.argv[2])
t = np.fromfile(sys.argv[1], np.uint64).astype(np.int64).reshape(-1, G, 16)[-1]
t = t[t[:, 11] > 0]
tree, tower, ev, it = t[:, 8], t[:, 9], t[:, 10], t[:, 11]
print("games %d, iterations/game %.0f, evals/game %.0f" % (len(t), it.mean(), ev.mean()))
print("tree phase  %8.0f cycles per simulation (p10 %.0f, p90 %.0f)" % ((tree / it).mean(), np.percentile(tree / it, 10), np.percentile(tree / it, 90)))
print("tower phase %8.0f cycles per evaluation (p10 %.0f, p90 %.0f)" % ((tower / np.maximum(ev, 1)).mean(), np.percentile(tower / np.maximum(ev, 1), 10), np.percentile(tower / np.maximum(ev, 1), 90)))
print("total       %8.0f cycles per simulation" % (((tree + tower) / it).mean()))

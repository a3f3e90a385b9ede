"""Phase stamps of the training Winograd convs (trace build: tools/build_variants.sh
trace=-DAZ_TOWER_TRACE, run with AZ_LIB=build_var/trace/libaz.so): per launch of
conv_wino_train_kernel in the last training step, the launch span and, per board (workgroup),
staging (entry -> staged barrier), core (-> wino_core done), epilogue (-> exit), in shader clocks,
and how busy the CUs were over the span.  20x256, batch 512, as tools/train_prof.py.
Usage: AZ_LIB=... python tools/train_trace.py [steps] [batch]   (batch <= 128: the part kernels, 4 or 2
workgroups per board: NP x B records per launch)"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "alphazero-chess_amd"))
import numpy as np
import azchess as A
from azchess import _lib as L

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
NP = 4 if 2 * B <= 256 else 1
rng = np.random.default_rng(1)
planes = (rng.random((B, 19, 64)) < 0.1).astype(np.float32)
pol = rng.random((B, 4096)).astype(np.float32)
pol /= pol.sum(1, keepdims=True)
val = rng.uniform(-1, 1, B).astype(np.float32)
tr = A.Trainer(20, 256, max_batch=B, seed=42)
rd = L.lib.az_train_trace_read
rd.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_int)]
n = C.c_int(0)
counts = []
for i in range(steps):
    tr.step(planes, pol, val, A.get_cyclical_lr(i))
    rd(None, 0, C.byref(n))
    counts.append(n.value)
per_step = counts[-1] - counts[-2]
print("Winograd training-conv launches per step:", per_step)
NL, NB = 128, 4096
buf = np.zeros(NL * NB * 8, np.uint64)
assert rd(buf.ctypes.data, buf.size, C.byref(n)) == 0
buf = buf.reshape(NL, NB, 8).astype(np.int64)
tot = {}
NW = NP * B                     # workgroups per launch (one board each, or NP parts of one)
for k in range(counts[-1] - per_step, counts[-1]):
    t = buf[k % NL, :NW]
    # each XCD has its own shader clock: the span per XCD, the longest
    span = max(t[t[:, 5] == x, 3].max() - t[t[:, 5] == x, 0].min() for x in np.unique(t[:, 5]))
    stage, core, epi = (t[:, 1] - t[:, 0]), (t[:, 2] - t[:, 1]), (t[:, 3] - t[:, 2])
    cu = (t[:, 5] << 16) | ((t[:, 4] >> 8) & 0xFF)      # XCC, SE / SH / CU of HW_ID
    ncu = len(np.unique(cu))
    busy = (t[:, 3] - t[:, 0]).sum() / (span * ncu)
    # boards per CU and the gap between a CU's consecutive boards
    order = np.lexsort((t[:, 0], cu))
    cs, ts, te = cu[order], t[order, 0], t[order, 3]
    same = cs[1:] == cs[:-1]
    gap = (ts[1:] - te[:-1])[same]
    # per CU: workgroup time over the union of its workgroups' intervals (how many were resident)
    conc = []
    for u in np.unique(cs):
        a_, b_ = ts[cs == u], te[cs == u]
        ev = np.concatenate([np.stack([a_, np.ones_like(a_)], 1), np.stack([b_, -np.ones_like(b_)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        lvl, last, busy_t = 0, 0, 0
        for tt, d in ev:
            if lvl > 0:
                busy_t += tt - last
            lvl += d
            last = tt
        conc.append((b_ - a_).sum() / max(busy_t, 1))
    cc = np.mean(conc)
    ph = "fwd" if k - (counts[-1] - per_step) < per_step // 2 else "bwd"
    print("launch %3d %s: span %7d  stage %6.0f core %6.0f epi %6.0f  CUs %3d  busy %.2f  gap %6.0f  resident %.2f"
          % (k, ph, span, stage.mean(), core.mean(), epi.mean(), ncu, busy, gap.mean() if gap.size else 0, cc))
    a = tot.setdefault(ph, np.zeros(5))
    a += [span, stage.mean(), core.mean(), epi.mean(), 1]
for ph, a in tot.items():
    s = a[:4] / a[4]
    print("%s mean: span %.0f  stage %.0f (%.1f%%)  core %.0f (%.1f%%)  epi %.0f (%.1f%%)  [2 x (stage+core+epi) = %.0f]"
          % (ph, s[0], s[1], 100 * s[1] / (s[1] + s[2] + s[3]), s[2], 100 * s[2] / (s[1] + s[2] + s[3]),
             s[3], 100 * s[3] / (s[1] + s[2] + s[3]), 2 * (s[1] + s[2] + s[3])))

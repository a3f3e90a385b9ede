"""Complete self-play games with the bench's net and search (20x256 random-init seed 42, 800
sims/move, Dirichlet noise, temperature moves, training.rs:294-378) until every game ends:
game-length distribution and the directly measured games/hr at this batch size.
Usage: python tools/game_length.py [games] [out.json] [f32|bf16]   (f32 = the headline's Winograd tower)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-chess_amd"))
import numpy as np  # noqa: E402

import azchess as A  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 256
out = sys.argv[2] if len(sys.argv) > 2 else None
dtype = sys.argv[3] if len(sys.argv) > 3 else "f32"
net = A.AlphaZero(20, 256, dtype=dtype, seed=42)
sp = A.SelfPlay(net, games=G, sims=800, continuous=False, seed=42, cache_capacity=0)
sp.reset()
t0 = time.perf_counter()
plies = {}
results = {}
moves = 0
while True:
    _, active = sp.step()
    moves += 1
    for st in sp.drain_raw():
        plies[st.game_id] = max(plies.get(st.game_id, 0), st.ply + 1)
        results[st.game_id] = st.result
    if moves % 20 == 0:
        print("move %d: %d active, %.0f s" % (moves, active, time.perf_counter() - t0), flush=True)
    if active == 0:
        break
dt = time.perf_counter() - t0
L = np.array(list(plies.values()))
st = sp.search.stats()
res = {"games": G, "sims_per_move": 800, "net": "20x256 %s random-init seed 42 (%s)" % (dtype, net.tower_kernel),
       "wall_s": dt,
       "games_per_hr_measured": G / dt * 3600, "sims_per_s": st["sims"] / dt,
       "plies_mean": float(L.mean()), "plies_median": float(np.median(L)), "plies_min": int(L.min()),
       "plies_max": int(L.max()),
       "results": {k: int(sum(1 for r in results.values() if r == v)) for k, v in
                   (("draw", 1), ("white", 2), ("black", 3))}}
print(json.dumps(res))
if out:
    with open(out, "w") as f:
        json.dump(res, f, indent=1)

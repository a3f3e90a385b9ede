"""C5 (BASELINE.json configs[4]) at its network size on one GPU: one iteration of train()
(training.rs:71-200 without the TUI / arena): 2048 concurrent self-play games of the 20x256 net at
f32 played to the end (sims/move reduced to --sims so the iteration fits one GPU call), the
replay buffer filled from their EpisodeSteps, then 40 AdamW steps on 512-position batches.
Prints one JSON line with the phase times, losses and replay growth.
Usage: python tools/c5_run.py [--games 2048] [--sims 32] [--min-replay 20000]"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-chess_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=2048)
ap.add_argument("--sims", type=int, default=32)
ap.add_argument("--blocks", type=int, default=20)
ap.add_argument("--filters", type=int, default=256)
ap.add_argument("--train-steps", type=int, default=40)
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--min-replay", type=int, default=20000)
ap.add_argument("--dtype", default="f32")
a = ap.parse_args()

import threading

import azchess as A

t0 = time.perf_counter()
stop = threading.Event()


def heartbeat():                                   # gpurun takes 3 silent minutes for a hang
    while not stop.wait(30):
        print("c5_run: %.0f s" % (time.perf_counter() - t0), file=sys.stderr, flush=True)


threading.Thread(target=heartbeat, daemon=True).start()
trainer, replay, hist = A.train(1, blocks=a.blocks, filters=a.filters, games=a.games, sims=a.sims,
                                min_replay=a.min_replay, train_steps=a.train_steps, batch_size=a.batch,
                                dtype=a.dtype)
wall = time.perf_counter() - t0
stop.set()
h = hist[0]
ok = math.isfinite(h["policy_loss"]) and math.isfinite(h["value_loss"]) and h["replay"] > 0
print(json.dumps({"config": "C5 (configs[4]) one iteration on 1 GPU: %d games x %d sims/move, %dx%d %s self-play, "
                            "%d train steps x %d" % (a.games, a.sims, a.blocks, a.filters, a.dtype, a.train_steps,
                                                     a.batch),
                  "wall_s": wall, "ok": ok, **h,
                  "selfplay_sims_per_s": h["selfplay_sims"] / h["selfplay_s"],
                  "train_ms_per_step": h["train_s"] / a.train_steps * 1e3}))
sys.exit(0 if ok else 1)

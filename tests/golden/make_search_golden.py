"""Generates tests/golden/search_c1.npz: search golden vectors (pin 4).

C1 of BASELINE.json (1 self-play game, 16 simulations per move) played to the end by the oracle's
restatement of run_episode / MCTree (training.rs:294-338, tree.rs:84-289), from startpos:
  * "synth": the synthetic evaluator (SplitMix64 of the position -> logits -> f32 softmax, value
    tanh of a hash-derived number; defined identically on the GPU side), Dirichlet noise on,
    seed 5, 2 games (game ids 0 and 1);
  * "net": the 2x32 network with the seeded random-init weights of tests/golden/net_2x32.npz,
    evaluated by the oracle's f32 network (agent.rs:112-144), noise on, seed 7, 1 game.
Per step: game, ply, chosen action (move index), search depth, result, final value, and the
root visit counts as CSR (vis_off, vis_idx, vis_n).  The reference itself cannot run here (Rust,
no toolchain), so these vectors pin the oracle against drift and the GPU path against a committed
fixture; parity with the reference stays unpinned.
Run:  python tests/golden/make_search_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

VARIANTS = {
    "synth": dict(sims=16, noise=True, seed=5, eval_kind=0, games=2, max_plies=0),
    "net": dict(sims=16, noise=True, seed=7, eval_kind=1, games=1, max_plies=0),
}


def run(name, net_weights=None):
    v = VARIANTS[name]
    net = O.RefNet(2, 32, net_weights) if v["eval_kind"] == 1 else None
    cfg = O.make_cfg(sims=v["sims"], noise=v["noise"], seed=v["seed"], eval_kind=v["eval_kind"], net=net)
    steps, sims, evals = O.selfplay(cfg, v["games"], max_plies=v["max_plies"])
    steps = sorted(steps, key=lambda s: (s["game"], s["ply"]))
    out = {k: np.array([s[k] for s in steps], np.float32 if k == "final_value" else np.int64)
           for k in ("game", "ply", "action", "depth", "result", "final_value")}
    off, idx, n = [0], [], []
    for s in steps:
        for k in sorted(s["visits"]):
            idx.append(k)
            n.append(s["visits"][k])
        off.append(len(idx))
    out["vis_off"] = np.array(off, np.int64)
    out["vis_idx"] = np.array(idx, np.int64)
    out["vis_n"] = np.array(n, np.float32)
    out["sims"] = np.array(sims, np.int64)
    out["evals"] = np.array(evals, np.int64)
    return {"%s_%s" % (name, k): a for k, a in out.items()}


def net_weights():
    return np.load(os.path.join(HERE, "net_2x32.npz"))["weights"].astype(np.float32)


def main():
    arrays = {}
    arrays.update(run("synth"))
    arrays.update(run("net", net_weights()))
    np.savez_compressed(os.path.join(HERE, "search_c1.npz"), **arrays)
    for k in ("synth", "net"):
        print(k, "steps", len(arrays[k + "_ply"]), "sims", int(arrays[k + "_sims"]), "evals", int(arrays[k + "_evals"]))


if __name__ == "__main__":
    main()

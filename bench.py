"""Benchmark: MCTS simulations/s of GPU-resident batched self-play (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): 2048 concurrent self-play games per GPU,
800 simulations per move, 20-block x 256-filter AlphaZero net (agent.rs), random-init
weights (seed 42), all games from the start position (training.rs:344-358).
One "step" = one move of every game = games x 800 simulations (select, expand, batched
network evaluation, backup) + action choice / play / re-root.  Games that end are
restarted in their slot, so every step does exactly games x sims simulations.
Multi-GPU: one process per GPU, games sharded (different seeds), no collective on the
path; barrier + max-over-ranks timing only.

Extra JSON fields: roofline (the residual 3x3 conv kernel vs bf16 dense MFMA peak,
measured with HIP events on the engine stream over the timed region), tree_walk (select
kernel, algorithmic bytes / time vs HBM peak), cpu_baseline (the oracle, rank 0, N=1,
bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "alphazero-chess_amd"))

PEAK_BF16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16
PEAK_F32_TFLOPS = 157.3       # MI355X_MICROARCH.md: f32 MFMA = vector peak
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: 8.0 TB/s spec
# HBM bytes per tower launch from rocprofv3 PMC passes (tools/pmc_run.sh: FETCH_SIZE x2 per the
# gfx950 correction + WRITE_SIZE), same kernel and per-launch work (2048 rows, 20x256 bf16)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_pmc_tower_v11_summary.json")
# mean plies of complete self-play games of this config (tools/game_length.py: 256 games, 20x256
# random-init seed 42, 800 sims/move, noise + temperature moves, played to the end)
GAME_LENGTH = os.path.join(ROOT, "profiles", "r01_game_length_256.json")


def pmc_traffic(games, blocks, filters, dtype):
    """Per-launch HBM traffic of the dominant kernel from the committed PMC summary, or None
    when the bench workload is not the one the counters were collected on."""
    if (games, blocks, filters, dtype) != (2048, 20, 256, "bf16") or not os.path.exists(PMC_SUMMARY):
        return None, None
    with open(PMC_SUMMARY) as f:
        s = json.load(f)
    return s.get("traffic_bytes"), os.path.relpath(PMC_SUMMARY, ROOT)


def cpu_baseline(blocks, filters, threads, games, sims):
    """Oracle (plain-C restatement of the reference, fp32) on the host cores: a bounded
    sample of the same workload -- `games` searches of `sims` simulations each from the
    start position with the same 20x256 net, one game per thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import azchess as A
    w = A.random_weights(blocks, filters, seed=42)
    net = O.RefNet(blocks, filters, w)
    cfg = O.make_cfg(sims=sims, noise=True, seed=42, eval_kind=1, net=net, threads=threads)
    t0 = time.perf_counter()
    steps, nsims, nevals = O.selfplay(cfg, games, max_plies=1)
    dt = time.perf_counter() - t0
    return {"value": nsims / dt, "unit": "sims/s", "cores": threads, "kind": "port",
            "sample": "%d games x 1 move x %d sims (+ shared root eval), %dx%d fp32 oracle, %d threads, %.1f s"
                      % (games, sims, blocks, filters, threads, dt),
            "evals": nevals}


def train_child(a):
    """`bench.py --train-child ...`: the training step (training.rs:147-190) on
    this rank's GPU, data-parallel over RCCL when world > 1 (gradients all-reduced over xGMI).
    Synthetic batch of BATCH_SIZE (512) positions per rank: random-playout planes, sparse visit
    policies, values in [-1, 1].  Prints one JSON line."""
    import numpy as np
    import azchess as A
    rng = np.random.default_rng(1234 + a.rank)
    B = a.train_batch
    planes = np.zeros((B, 19, 64), np.float32)
    for i in range(B):                         # piece-like one-hot planes + constant planes
        sq = rng.permutation(64)[:int(rng.integers(4, 32))]
        planes[i, rng.integers(0, 12, len(sq)), sq] = 1.0
        planes[i, 12:16] = rng.integers(0, 2, (4, 1))
        planes[i, 17] = rng.integers(0, 100) / 100.0
        planes[i, 18] = rng.integers(1, 200) / 200.0
    pol = np.zeros((B, 4096), np.float32)
    for i in range(B):
        idx = rng.choice(4096, 30, replace=False)
        v = rng.integers(1, 40, 30).astype(np.float32)
        pol[i, idx] = v / v.sum()
    val = rng.uniform(-1, 1, B).astype(np.float32)
    tr = A.Trainer(a.blocks, a.filters, max_batch=B, device=a.device, seed=42)
    if a.world > 1:
        tr.set_comm(bytes.fromhex(a.uid), a.rank, a.world)
    for it in range(2):
        tr.step(planes, pol, val, A.get_cyclical_lr(it))
    tr.timing(reset=True)
    t0 = time.perf_counter()
    for it in range(a.train_steps):
        tr.step(planes, pol, val, A.get_cyclical_lr(it))
    wall = (time.perf_counter() - t0) / a.train_steps
    dev_ms, ar_ms, n = tr.timing()
    print(json.dumps({"ms_per_step": wall * 1e3, "device_ms_per_step": dev_ms / n, "allreduce_ms_per_step": ar_ms / n}))


def train_phase(args, A, rank, world, local):
    """Run train_child on every rank (subprocess with a time limit, so a collective that never
    completes cannot hold the self-play measurement hostage); rank 0 returns the summary."""
    import subprocess
    uid = ""
    if world > 1:
        import torch.distributed as dist
        box = [A.comm_unique_id().hex() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    cmd = [sys.executable, os.path.abspath(__file__), "--train-child", "--rank", str(rank), "--world", str(world),
           "--device", str(local), "--uid", uid or "-", "--blocks", str(args.blocks), "--filters", str(args.filters),
           "--train-steps", str(args.train_steps), "--train-batch", str(args.train_batch)]
    res, err = None, None
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=args.train_timeout)
        lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if out.returncode == 0 and lines:
            res = json.loads(lines[-1])
        else:
            err = "rc %d: %s" % (out.returncode, (out.stderr or out.stdout)[-400:])
    except subprocess.TimeoutExpired:
        err = "timed out after %d s" % args.train_timeout
    ms = res["ms_per_step"] if res else float("nan")
    if world > 1:
        import torch
        import torch.distributed as dist
        t = torch.tensor([ms if res else float("inf")], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    if rank != 0:
        return None
    flop = 3.0 * net_flop_per_eval(args.blocks, args.filters) * args.train_batch
    out = {"what": "training.rs:147-190 step: training-mode forward + backward + clip + AdamW, f32 "
                   "(v_mfma_f32_16x16x4_f32), %d positions per rank%s" %
                   (args.train_batch, ", gradients all-reduced over RCCL" if world > 1 else ""),
           "global_batch": args.train_batch * world, "dtype": "f32"}
    if res and ms == ms and ms != float("inf"):
        tf = flop / (res["device_ms_per_step"] * 1e-3) / 1e12
        out.update({"ms_per_step": ms, "samples_per_s": args.train_batch * world / (ms * 1e-3),
                    "device_ms_per_step": res["device_ms_per_step"],
                    "allreduce_ms_per_step": res["allreduce_ms_per_step"],
                    "allreduce_bytes": 4 * int(A._lib.lib.az_net_num_params(args.blocks, args.filters)),
                    "achieved_tflops": tf, "peak_tflops": PEAK_F32_TFLOPS, "frac": tf / PEAK_F32_TFLOPS,
                    "flop_per_step": flop})
    else:
        out["error"] = err or "a rank failed"
    return out


def net_flop_per_eval(B, F):
    """forward FLOPs per position"""
    return 2.0 * 64.0 * (171.0 * F + 18.0 * B * F * F + 40.0 * F + 2048.0) + 2.0 * (32768.0 + 64.0)


def config_name(games, sims, blocks, filters):
    """Which BASELINE.json config this run is: C3 = configs[2] (the headline), C2 = configs[1]."""
    if (sims, blocks, filters) == (800, 20, 256) and games == 2048:
        return "C3 (BASELINE.json configs[2])"
    if (sims, blocks, filters) == (800, 6, 64) and games == 256:
        return "C2 (BASELINE.json configs[1])"
    return "custom (not a BASELINE.json config)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--games", type=int, default=2048)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--filters", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cache", type=int, default=500000, help="FEN cache entries (CACHE_CAPACITY, 0 = off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-games", type=int, default=16)
    ap.add_argument("--cpu-sims", type=int, default=32, help="sims per sampled search (~12 s of host work at 20x256)")
    ap.add_argument("--train-steps", type=int, default=5, help="timed training steps (0 = skip the training phase)")
    ap.add_argument("--train-batch", type=int, default=512, help="positions per rank (BATCH_SIZE, parameters.rs:17)")
    ap.add_argument("--train-timeout", type=int, default=240)
    ap.add_argument("--train-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--uid", default="-", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.train_child:
        return train_child(args)

    # libaz (and the /opt/rocm HIP runtime it is built for) is loaded before torch: torch
    # bundles its own libamdhip64.so.7 (same SONAME) and is only used here for the gloo
    # barrier / reduction between ranks -- the self-play path has no collective.
    import azchess as A
    from azchess.dist import barrier as dist_barrier, env_rank, reduce_run, shard
    rank, world, local = env_rank()
    import ctypes
    ndev = ctypes.c_int(0)
    A._lib.lib.az_device_count(ctypes.byref(ndev))
    if ndev.value < 1:
        raise SystemExit("bench.py: no GPU visible to libaz")
    local = local % ndev.value          # one GPU per rank; wraps only when rehearsing on fewer GPUs
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    G, S = args.games, args.sims
    net = A.AlphaZero(args.blocks, args.filters, dtype=args.dtype, device=local, seed=42)
    sh = shard(rank, world, G)

    def synchronize():
        A._lib.check(A._lib.lib.az_device_synchronize(local))

    def barrier():
        dist_barrier(world)
        synchronize()

    def phase(cache, steps, timing):
        """Self-play from startpos: warmup moves, then `steps` timed moves of every game."""
        sp = A.SelfPlay(net, games=G, sims=S, device=local, continuous=True, seed=sh["seed"], cache_capacity=cache)
        sp.reset()
        for _ in range(args.warmup):
            sp.step()
            sp.drain()
        st0 = sp.search.stats()
        sp.search.timing(reset=True, enable=timing)
        barrier()
        t0 = time.perf_counter()
        finished = 0
        for _ in range(steps):
            f, _ = sp.step()
            finished += f
            sp.drain()
        synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        tm = sp.search.timing(reset=False, enable=False)
        st1 = sp.search.stats()
        c = [st1[k] - st0[k] for k in ("sims", "evals", "terminal_leaves", "moves", "max_depth_sum", "cache_hits")]
        assert c[0] == G * S * steps, (c[0], G * S * steps)
        elapsed, tot = reduce_run(elapsed, c + [finished], world)
        del sp
        return elapsed, dict(zip(("sims", "evals", "terminal", "moves", "depth", "hits", "finished"), tot)), tm, c[0]

    # headline: no FEN cache -> every non-terminal simulation evaluates its leaf on the network
    elapsed, tot, tm, sims_rank = phase(0, args.steps, True)
    sims_all, evals_all, term_all = tot["sims"], tot["evals"], tot["terminal"]
    fin_all, moves_all, depth_all = tot["finished"], tot["moves"], tot["depth"]
    # the reference's FEN cache (tree.rs:214-219, CACHE_CAPACITY = 500k) on the same window
    cache_res = None
    if args.cache > 0:
        e2, t2, _, _ = phase(args.cache, args.steps, False)
        cache_res = {"value": t2["sims"] / e2, "unit": "sims/s", "evals_per_sim": t2["evals"] / max(t2["sims"], 1),
                     "cache_hit_frac": t2["hits"] / max(t2["sims"], 1), "entries": args.cache,
                     "note": "same window with the reference's FEN evaluation cache (A12); games are in "
                             "lockstep from startpos, so early moves share most positions"}

    training = train_phase(args, A, rank, world, local) if args.train_steps > 0 else None
    if rank != 0:
        dist.destroy_process_group()
        return
    value = sims_all / elapsed
    traffic, traffic_src = pmc_traffic(G, args.blocks, args.filters, args.dtype)
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    conv_tflops = tm["conv_flop"] / (tm["conv_ms"] * 1e-3) / 1e12 if tm["conv_ms"] > 0 else 0.0
    tower_tflops = tm["tower_flop"] / (tm["tower_ms"] * 1e-3) / 1e12 if tm["tower_ms"] > 0 else 0.0
    # select_bytes covers every k_select launch of the window (steps x S); the event times cover
    # the sampled launches (az_timing: every 8th simulation step)
    sel_bytes_per_launch = tm["select_bytes"] / max(args.steps * S, 1)
    sel_ms_per_launch = tm["select_ms"] / max(tm["select_launches"], 1)
    sel_gbs = sel_bytes_per_launch / (sel_ms_per_launch * 1e-3) / 1e9 if tm["select_ms"] > 0 else 0.0
    out = {
        "metric": "MCTS sims/sec at 800 sims/move, 20x256 net; self-play games/hr at 1/2/4/8 GPU",
        "value": value,
        "unit": "sims/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic: random-init %dx%d weights (seed 42), self-play from startpos, Dirichlet noise on"
                % (args.blocks, args.filters),
        "config": {"workload": "%s: %d concurrent self-play games/GPU x %d sims/move, %d-block x %d-filter net"
                               % (config_name(G, S, args.blocks, args.filters), G, S, args.blocks, args.filters),
                   "games_per_gpu": G, "sims_per_move": S, "blocks": args.blocks, "filters": args.filters,
                   "fen_cache": "off for value (see with_fen_cache)",
                   "parallelism": "games sharded %d-way, no collective (gloo barrier/max only)" % world},
        "roofline": {"bound": "mfma", "achieved": conv_tflops, "peak": peak, "unit": "TFLOP/s",
                     "frac": conv_tflops / peak, "traffic": traffic,
                     "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                     "kernel": ("tower_kernel<%d> (fused input conv + %d residual convs + heads; algorithmic "
                                "FLOPs = conv FLOPs only), %d launches timed (HIP events on every 8th simulation step)" % (args.filters, 2 * args.blocks,
                                                                                 tm["conv_launches"]))
                               if net.fused_tower else
                               "conv3x3_kernel<%d,%d> (residual 3x3 conv), %d launches timed" %
                               (args.filters, args.filters, tm["conv_launches"]),
                     "flop_per_launch": tm["conv_flop"] / max(tm["conv_launches"], 1),
                     "avg_ms_per_launch": tm["conv_ms"] / max(tm["conv_launches"], 1)},
        "tower": {"achieved_tflops": tower_tflops, "frac": tower_tflops / peak,
                  "ms_per_sim_step": tm["tower_ms"] / max(tm["sim_steps"], 1)},
        "tree_walk": {"kernel": "k_select", "achieved_gbs": sel_gbs, "peak_gbs": PEAK_HBM_GBS,
                      "frac": sel_gbs / PEAK_HBM_GBS,
                      "bytes_per_sim": tm["select_bytes"] / max(sims_rank, 1),
                      "avg_ms_per_launch": tm["select_ms"] / max(tm["select_launches"], 1)},
        "sim_step_ms": {k: tm[k + "_ms"] / max(tm["sim_steps"], 1)
                        for k in ("select", "expand", "encode", "tower", "heads", "backup")},
        "evals_per_sim": evals_all / max(sims_all, 1),
        "terminal_leaf_frac": term_all / max(sims_all, 1),
        "with_fen_cache": cache_res,
        "avg_search_depth": depth_all / max(moves_all, 1),
        "games_finished": int(fin_all),
        "games_per_hr": fin_all / elapsed * 3600.0,
        "games_per_hr_projected": None,
        "cpu_baseline": None,
        "training": training,
    }
    if (args.blocks, args.filters, S) == (20, 256, 800) and os.path.exists(GAME_LENGTH):
        with open(GAME_LENGTH) as f:
            gl = json.load(f)
        # continuous self-play keeps every slot busy (a finished game restarts in its slot), so
        # the steady state plays sims/s / (sims/move * plies/game) games
        out["games_per_hr_projected"] = {
            "value": value * 3600.0 / (S * gl["plies_mean"]), "plies_per_game": gl["plies_mean"],
            "source": os.path.relpath(GAME_LENGTH, ROOT),
            "note": "steady-state continuous self-play: measured sims/s / (800 sims x mean plies of %d complete "
                    "games); the timed window is %d moves, too short for games to finish" % (gl["games"], args.steps)}
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.blocks, args.filters, args.cpu_threads, args.cpu_games,
                                           args.cpu_sims)
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Benchmark: MCTS simulations/s of GPU-resident batched self-play (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): 2048 concurrent self-play games per GPU,
800 simulations per move, 20-block x 256-filter AlphaZero net (agent.rs), random-init
weights (seed 42), all games from the start position (training.rs:344-358), evaluated in
f32 like the reference (burn Cuda<f32>, main.rs:15,68).
One "step" = `--sims-per-step` (default 100) simulation steps of every game, i.e. games x 100
simulations (select, expand, batched network evaluation, backup); every 8th step completes a
move (800 sims), whose action choice / play / re-root fall inside that step.  Games that end
are restarted in their slot, so every step does exactly games x sims-per-step simulations.
Multi-GPU: one process per GPU (torchrun, or `--gpus N` spawns the N ranks itself), games
sharded (different seeds), no collective on the path; barrier + max-over-ranks timing only.

Extra JSON fields: roofline (the fused tower kernel vs the f32 MFMA peak, HIP events on the
engine stream over the timed region), bf16_mode (the same window with the bf16 tower, labelled,
with its stated tolerance), tree_walk (select kernel, algorithmic bytes / time vs HBM peak),
c2_steady (configs[1] in steady state: 256 games, 6x64 f32, with its tower roofline),
games_per_hr_measured (C2's games played to the end), cpu_baseline (the oracle, rank 0, N=1,
bounded sample), training (the C5 gradient step, per-rank and sharded-batch modes).
`--rehearse` runs the multi-rank plumbing with a CPU stub engine (no GPU; CI only).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "alphazero-chess_amd"))

PEAK_BF16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16
PEAK_F32_TFLOPS = 157.3       # MI355X_MICROARCH.md: f32 MFMA = vector peak
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: 8.0 TB/s spec
# HBM bytes per tower launch from rocprofv3 PMC passes (tools/pmc_run.sh: FETCH_SIZE x2 per the
# gfx950 correction + WRITE_SIZE), same kernel and per-launch work (2048 rows, 20x256)
PMC_SUMMARY = {"f32": os.path.join(ROOT, "profiles", "r06_pmc_tower32w_summary.json"),             # Winograd
               "f32-direct": os.path.join(ROOT, "profiles", "r02_pmc_tower32_summary.json"),      # AZ_WINOGRAD=0
               "bf16": os.path.join(ROOT, "profiles", "r04_pmc_tower_bf16_summary.json")}
# simulation steps of the instrumented profile pass after the timed window (8 sampled tower launches)
PROFILE_SIMS = 256
# mean plies of complete self-play games of this config (tools/game_length.py: 256 games, 20x256
# random-init seed 42, 800 sims/move, noise + temperature moves, played to the end)
# (f32 Winograd net, the headline's; the round-1 file used the bf16 net and is only a fallback)
GAME_LENGTH = [os.path.join(ROOT, "profiles", "r03_game_length_c3_f32.json"),
               os.path.join(ROOT, "profiles", "r01_game_length_256.json")]
# stated tolerances of the two tower precisions against the f32 oracle (tests/test_gpu_net.py)
TOLERANCE = {"f32": "value |d| <= 1e-5, policy |d| <= 1e-4 p + 1e-8 (tests/test_gpu_net.py)",
             "bf16": "value |d| <= 2e-2, policy |d| <= 5e-2 p + 2e-5, total variation <= 2e-2 "
                     "(tests/test_gpu_net.py)"}


def pmc_traffic(games, blocks, filters, dtype, winograd=True):
    """Per-launch HBM traffic of the dominant kernel from the committed PMC summary, or None
    when the bench workload is not the one the counters were collected on."""
    path = PMC_SUMMARY.get(dtype if dtype != "f32" or winograd else "f32-direct")
    if (games, blocks, filters) != (2048, 20, 256) or not path or not os.path.exists(path):
        return None, None
    with open(path) as f:
        s = json.load(f)
    return s.get("traffic_bytes"), os.path.relpath(path, ROOT)


def cgroup_cpus():
    """The CPUs the process's cgroup may use (cgroup v2 cpu.max quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        pass
    try:   # cgroup v1
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = float(f.read())
        return q / p if q > 0 and p > 0 else None
    except (OSError, ValueError):
        return None


def cpu_baseline(blocks, filters, threads, games, sims, port=True):
    """The reference's self-play on the host cores, a bounded sample of the same workload: `games`
    games from the start position, one move of `sims` simulations each, same 20x256 net (seed 42).
    Batched like the reference's batcher (training.rs:340-422): the oracle's trees (dense 4096
    arrays, state clone per node, tree.rs) step in lockstep, OpenMP over games, and every
    simulation step evaluates all pending leaves in ONE f32 forward through torch-CPU's oneDNN
    convolutions (oracle/cpu_net.py: BN folded, channels-last, `threads` OpenMP threads).  Beside
    it, the per-game port (one leaf at a time, naive C convolution) of earlier rounds."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import azchess as A
    from cpu_net import CpuNet
    w = A.random_weights(blocks, filters, seed=42)
    net = CpuNet(blocks, filters, w, threads=threads)
    net.forward(np.zeros((games, 19, 8, 8), np.float32))          # warm oneDNN's kernels
    cfg = O.make_cfg(sims=sims, noise=True, seed=42, eval_kind=1, threads=threads)
    t0 = time.perf_counter()
    steps, nsims, nevals = O.selfplay_batched(cfg, games, max_plies=1, evaluator=net.forward)
    dt = time.perf_counter() - t0
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), None)
    except OSError:
        pass
    out = {"value": nsims / dt, "unit": "sims/s", "kind": "port",
           "cores": os.cpu_count(), "nproc": len(os.sched_getaffinity(0)), "threads": threads,
           "cpu_quota": cgroup_cpus(),
           "cores_note": "cores = os.cpu_count() of the GPU box's host, nproc = the CPUs this process may run on "
                         "(the box's share), threads = the OpenMP / torch threads the baseline used",
           "cpu_model": model,
           "conv_algorithm": "oneDNN brg_conv_fwd:avx512_core, alg:convolution_direct (ONEDNN_VERBOSE=1 on the 3x3 "
                             "and 1x1 convs of oracle/cpu_net.py: direct brgemm convolution, no Winograd)",
           "sample": "%d games x 1 move x %d sims (+ shared root eval) in lockstep, one batched f32 forward per "
                     "simulation step (torch-CPU oneDNN, BN folded), %dx%d net, %d threads, %.1f s"
                     % (games, sims, blocks, filters, threads, dt),
           "evals": nevals}
    if not port:
        return out
    rnet = O.RefNet(blocks, filters, w)
    psims = max(sims // 16, 1)
    pcfg = O.make_cfg(sims=psims, noise=True, seed=42, eval_kind=1, net=rnet, threads=threads)
    t0 = time.perf_counter()
    _, pdone, _ = O.selfplay(pcfg, 16, max_plies=1)
    pdt = time.perf_counter() - t0
    out["per_game_port"] = {"value": pdone / pdt, "unit": "sims/s", "threads": threads,
                            "sample": "16 games x 1 move x %d sims, one leaf per game at a time, naive C "
                                      "convolution (oracle/net_ref.c), %.1f s" % (psims, pdt)}
    return out


def train_child(a):
    """`bench.py --train-child ...`: the training step (training.rs:147-190) on
    this rank's GPU, data-parallel over RCCL when world > 1 (gradients all-reduced over xGMI).
    Synthetic batch of BATCH_SIZE (512) positions per rank: random-playout planes, sparse visit
    policies, values in [-1, 1].  Prints one JSON line."""
    import numpy as np
    import azchess as A
    rng = np.random.default_rng(1234 + (0 if a.train_mode == "sharded" else a.rank))
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
    sharded = a.train_mode == "sharded"
    if sharded:      # this rank's shard of the one global batch (every rank generated all of it)
        from azchess.training import shard_bounds
        lo, hi = shard_bounds(B, a.rank, a.world)
        if hi <= lo:
            raise SystemExit("--train-batch %d leaves rank %d no rows" % (B, a.rank))
        B = hi - lo
        planes, pol, val = planes[lo:hi], pol[lo:hi], val[lo:hi]
    tr = A.Trainer(a.blocks, a.filters, max_batch=B, device=a.device, seed=42)
    if a.world > 1 or sharded:     # sharded at world 1: the 1-rank communicator, so its collectives are timed
        tr.set_comm(bytes.fromhex(a.uid) if a.uid != "-" else A.comm_unique_id(), a.rank, a.world)
    tr.set_sharded(sharded)
    for it in range(2):
        tr.step(planes, pol, val, A.get_cyclical_lr(it))
    tr.timing(reset=True)
    tr.exchange_stats(reset=True)
    t0 = time.perf_counter()
    for it in range(a.train_steps):
        tr.step(planes, pol, val, A.get_cyclical_lr(it))
    wall = (time.perf_counter() - t0) / a.train_steps
    dev_ms, ar_ms, n = tr.timing()
    nx, nxs, _ = tr.exchange_stats(reset=True)
    xms = None
    if nx:    # the exchanges' own time in separate steps (their events cost queue time)
        tr.time_exchanges(True)
        for it in range(a.train_steps):
            tr.step(planes, pol, val, A.get_cyclical_lr(it))
        _, xs, xt = tr.exchange_stats()
        xms = xt / max(xs, 1)
    print(json.dumps({"ms_per_step": wall * 1e3, "device_ms_per_step": dev_ms / n, "allreduce_ms_per_step": ar_ms / n,
                      "rows": B, "collectives_per_step": nx / max(nxs, 1), "exchange_ms_per_step": xms}))


def train_phase(args, A, rank, world, local, mode="per-rank"):
    """Run train_child on every rank (subprocess with a time limit, so a collective that never
    completes cannot hold the self-play measurement hostage); rank 0 returns the summary.
    mode "per-rank": every rank trains its own --train-batch positions (global batch x world, per-rank
    BatchNorm); "sharded": the reference's ONE batch of --train-batch split over the ranks, BatchNorm
    statistics exchanged over RCCL (az_trainer_set_sharded)."""
    uid = ""
    sharded = mode == "sharded"
    if world > 1 or sharded:
        import torch.distributed as dist
        if world > 1:
            box = [A.comm_unique_id().hex() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        else:
            uid = A.comm_unique_id().hex()
    cmd = [sys.executable, os.path.abspath(__file__), "--train-child", "--rank", str(rank), "--world", str(world),
           "--device", str(local), "--uid", uid or "-", "--blocks", str(args.blocks), "--filters", str(args.filters),
           "--train-steps", str(args.train_steps), "--train-batch", str(args.train_batch), "--train-mode", mode]
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
    gb = args.train_batch if sharded else args.train_batch * world     # global batch
    lb = -(-gb // world)             # positions of the largest shard (sharded: ranks get floor / ceil)
    flop = 3.0 * net_flop_per_eval(args.blocks, args.filters) * lb
    # executed MFMA work: the residual convs of forward, data grad and weight grad run as Winograd
    # F(2x2,3x3) at F = 256 (train.hip; AZ_TRAIN_WINOGRAD=0 restores direct convs)
    wino = args.filters == 256 and os.environ.get("AZ_TRAIN_WINOGRAD", "1") != "0"
    xflop = 3.0 * executed_flop_per_eval(args.blocks, args.filters, wino) * lb
    out = {"what": "training.rs:147-190 step: training-mode forward + backward + clip + AdamW, f32 "
                   "(v_mfma_f32_16x16x4_f32), %d positions per rank%s" %
                   (lb, ", gradients all-reduced over RCCL" if world > 1 else ""),
           "mode": mode,
           "mode_note": ("the reference's one batch of %d split over %d rank(s); every BatchNorm's batch statistics "
                         "and backward sums all-reduced over RCCL (2 collectives per tower BN, one per direction for "
                         "the two head BNs together, the losses inside the gradient all-reduce) -- bit-identical to "
                         "the per-rank step at world 1; exchange_ms_per_step times every collective (HIP events on "
                         "the trainer stream), allreduce_ms_per_step the gradient's alone" % (gb, world))
                        if sharded else
                        ("%d positions per rank, per-rank BatchNorm statistics, gradients averaged over ranks "
                         "(global batch %d)" % (lb, gb)),
           "global_batch": gb, "dtype": "f32"}
    if res and ms == ms and ms != float("inf"):
        tf = xflop / (res["device_ms_per_step"] * 1e-3) / 1e12
        out.update({"ms_per_step": ms, "samples_per_s": gb / (ms * 1e-3),
                    "device_ms_per_step": res["device_ms_per_step"],
                    "allreduce_ms_per_step": res["allreduce_ms_per_step"],
                    "rows_rank0": res.get("rows"), "collectives_per_step": res.get("collectives_per_step"),
                    "exchange_ms_per_step": res.get("exchange_ms_per_step"),
                    "allreduce_bytes": 4 * int(A._lib.lib.az_net_num_params(args.blocks, args.filters)),
                    "achieved_tflops": tf, "peak_tflops": PEAK_F32_TFLOPS, "frac": tf / PEAK_F32_TFLOPS,
                    "executed_flop_per_step": xflop, "residual_convs": "winograd" if wino else "direct",
                    "algorithmic_flop_per_step": flop,
                    "algorithmic_tflops": flop / (res["device_ms_per_step"] * 1e-3) / 1e12,
                    "algorithmic_note": "3 x the direct-conv forward FLOPs (SURVEY 8a A6) / device time: "
                                        "an equivalent rate, not a fraction of a peak"})
    else:
        out["error"] = err or "a rank failed"
    return out


def net_flop_per_eval(B, F):
    """forward FLOPs per position"""
    return 2.0 * 64.0 * (171.0 * F + 18.0 * B * F * F + 40.0 * F + 2048.0) + 2.0 * (32768.0 + 64.0)


def executed_flop_per_eval(B, F, winograd):
    """The forward's FLOPs as the training kernels issue them: the 2B residual 3x3 convs as Winograd
    F(2x2,3x3) (16 points x 16 tiles x F^2 multiply-adds per conv instead of 64 squares x 9 taps),
    everything else direct"""
    direct = net_flop_per_eval(B, F)
    if not winograd:
        return direct
    resid = 2.0 * 64.0 * 18.0 * B * F * F
    return direct - resid + 2.0 * (2 * B) * 256.0 * F * F


def tower_algo_flop_per_row(B, F):
    """algorithmic (direct-conv) FLOPs the engine books per evaluated row (az_timing.conv_flop):
    input conv + 2B residual 3x3 convs, SURVEY 8a A6 without the heads"""
    return 2.0 * 64.0 * (171.0 * F + 18.0 * B * F * F)


def tower_exec_flop_per_row(B, F, dtype, wino):
    """MFMA FLOPs the fused tower issues per row: the input conv (direct towers: 19 input planes
    padded to 32 channels, 18 k-steps of 16; Winograd towers: channels 16-18 of four taps packed per
    k-step, 12 k-steps of 16 -- tower.hip conv32_in_packed), the residual convs (Winograd: 16 points x 16 tiles x F x F per conv; direct: 64
    squares x 9 taps x F x F), the heads' 1x1 F->40 conv padded to 48 rows (bf16 mode: split into
    hi + lo bf16 fragments, twice the MFMAs) and the 32->64 policy conv.  The value MLP runs on
    VALU.  Cross-check: PMC SQ_INSTS_MFMA x 2048 FLOP (profiles/*pmc*summary.json)."""
    res = (16.0 * 16.0 if (wino and dtype != "bf16") else 64.0 * 9.0) * 2.0 * F * F * 2 * B
    heads = 2.0 * 64.0 * 48.0 * F * (2 if dtype == "bf16" else 1) + 2.0 * 64.0 * 64.0 * 32.0
    inconv = 2.0 * 64.0 * 16.0 * (12.0 if (wino and dtype != "bf16") else 18.0) * F
    return inconv + res + heads


def config_name(games, sims, blocks, filters):
    """Which BASELINE.json config this run is: C3 = configs[2] (the headline), C2 = configs[1]."""
    if (sims, blocks, filters) == (800, 20, 256) and games == 2048:
        return "C3 (BASELINE.json configs[2])"
    if (sims, blocks, filters) == (800, 6, 64) and games == 256:
        return "C2 (BASELINE.json configs[1])"
    return "custom (not a BASELINE.json config)"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def auto_sims_per_step(S, steps, warmup):
    """Bench step size: the smallest divisor K >= 40 of S (or S) with steps*K and warmup*K whole
    moves, so the timed window starts at a move boundary and carries its share of move completions
    (k_finish, EpisodeStep drain, re-root); 100 if none (then window_move_aligned = false)."""
    for K in range(min(40, S), S + 1):
        if S % K == 0 and (steps * K) % S == 0 and (warmup * K) % S == 0:
            return K
    return 100 if S % 100 == 0 else S


def play_games_leg(A, device, seed, world, barrier, synchronize, games=256, sims=800, blocks=6, filters=64):
    """C2 (BASELINE.json configs[1]: 256 games x 800 sims/move, 6x64 f32 net) from startpos until
    every game has ended (run_all_episodes, training.rs:340-378): completed games / wall time of
    the slowest rank.  A measurement, not a projection; the C3 headline's games/hr is projected
    (a C3 game at 800 sims takes tens of minutes)."""
    from azchess.dist import reduce_run
    net = A.AlphaZero(blocks, filters, dtype="f32", device=device, seed=42)
    sp = A.SelfPlay(net, games=games, sims=sims, device=device, continuous=False, seed=seed + 7, cache_capacity=0)
    sp.reset()
    barrier()
    t0 = time.perf_counter()
    while True:
        _, active = sp.step()
        sp.drain_raw()                 # EpisodeSteps leave the engine as in the reference (memory.rs input)
        if active == 0:
            break
    synchronize()
    barrier()
    dt = time.perf_counter() - t0
    st = sp.search.stats()
    dt_max, tot = reduce_run(dt, [st["games_finished"], st["moves"], st["sims"]], world)
    del sp, net
    return {"value": tot[0] / dt_max * 3600.0, "unit": "games/hr", "games": int(tot[0]),
            "plies_mean": tot[1] / max(tot[0], 1), "wall_s": dt_max, "sims_per_s": tot[2] / dt_max,
            "config": "C2 (BASELINE.json configs[1]): %d games/GPU x %d sims/move, %dx%d f32 net, played from "
                      "startpos to the end (not continuous: the batch shrinks as games end)" % (games, sims, blocks, filters)}


def launch_ranks(n):
    """`bench.py --gpus N` without a torchrun environment: start N fresh child processes of this
    script, one per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1), and exit
    with the worst child status.  Runs before anything touches the GPU (no exec: children)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll: a rank that dies before the rendezvous must not leave its siblings blocked in
    # init_process_group for gloo's default timeout -- terminate them and return its status
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


class _RehearsalSearch:
    """Counters / timing of the CPU stub engine (same keys as BatchedSearch)."""

    def __init__(self, games):
        self.games = games
        self.c = dict(sims=0, evals=0, terminal_leaves=0, moves=0, max_depth_sum=0, cache_hits=0)

    def stats(self):
        return dict(self.c)

    def timing(self, reset=False, enable=None):
        keys = ("select", "expand", "encode", "tower", "heads", "backup", "conv")
        t = {k + "_ms": 0.0 for k in keys}
        t.update(conv_flop=0.0, tower_flop=0.0, conv_launches=0, select_launches=0, sim_steps=0, select_bytes=0.0)
        return t


class RehearsalSelfPlay:
    """`--rehearse`: a CPU stand-in for azchess.SelfPlay with the same interface, so the multi-rank
    plumbing of bench.py (spawn, per-rank seeds, barrier, max-over-ranks, counter sums, JSON line)
    runs in a container without a GPU.  It does a little numpy work per simulation step; its
    numbers measure nothing and are labelled as such."""

    def __init__(self, games, sims, seed):
        import numpy as np
        self.np, self.games, self.S = np, games, sims
        self.rng = np.random.default_rng(seed)
        self.search = _RehearsalSearch(games)
        self.cursor = 0

    def reset(self):
        self.cursor = 0

    def run_sims(self, n):
        n = min(n, self.S - self.cursor)
        a = self.rng.standard_normal((64, 64)).astype(self.np.float32)
        for _ in range(n):
            a = self.np.tanh(a @ a.T * 1e-2)
        self.cursor += n
        self.search.c["sims"] += self.games * n
        self.search.c["evals"] += self.games * n
        done = self.cursor == self.S
        if done:
            self.cursor = 0
            self.search.c["moves"] += self.games
        return 0, (self.games if done else -1), done

    def drain(self):
        return []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--games", type=int, default=2048)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--sims-per-step", type=int, default=0,
                    help="simulation steps of every game per bench step (0 = auto: the smallest divisor of "
                         "--sims >= 40 that makes the warmup and the timed window whole moves)")
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--filters", type=int, default=256)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                    help="headline precision (the reference computes in f32)")
    ap.add_argument("--c2-steps", type=int, default=20,
                    help="moves (800 sims each) of the C2 steady-state leg: 256 games x 6x64 f32 (0 = skip)")
    ap.add_argument("--bf16-steps", type=int, default=-1,
                    help="steps of the labelled bf16_mode leg (-1 = same as --steps, 0 = skip)")
    ap.add_argument("--cache", type=int, default=0,
                    help="FEN cache entries for an extra with_fen_cache leg (CACHE_CAPACITY = 500000; 0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-games", type=int, default=64)
    ap.add_argument("--cpu-sims", type=int, default=160, help="sims per sampled search (batched leg ~8 s of host work at 20x256 on 16 threads)")
    ap.add_argument("--train-steps", type=int, default=5, help="timed training steps (0 = skip the training phase)")
    ap.add_argument("--train-batch", type=int, default=512, help="positions per rank (BATCH_SIZE, parameters.rs:17)")
    ap.add_argument("--train-timeout", type=int, default=90)
    ap.add_argument("--train-mode", default="per-rank", choices=["per-rank", "sharded"], help=argparse.SUPPRESS)
    ap.add_argument("--games-leg", type=int, default=1,
                    help="1: also play C2's games (256 x 800 sims, 6x64 f32) from startpos to the end on every rank "
                         "and report the measured games/hr (0 = skip); its wall time is in legs_wall_s")
    ap.add_argument("--same-device", action="store_true",
                    help="test only: every rank runs on device 0 and the RCCL training leg is skipped (exercises the "
                         "N>1 rank path with the real engine on a 1-GPU box; not a scaling measurement)")
    ap.add_argument("--rehearse", action="store_true",
                    help="no GPU: run the rank plumbing with a CPU stub engine (gloo); numbers are meaningless")
    ap.add_argument("--train-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--uid", default="-", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.train_child:
        return train_child(args)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)

    from azchess.dist import barrier as dist_barrier, env_rank, reduce_run, shard
    rank, world, local = env_rank()
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    G, S, K = args.games, args.sims, args.sims_per_step
    if K == 0:
        K = auto_sims_per_step(S, args.steps, args.warmup)
    if K < 1 or S % K:
        raise SystemExit("bench.py: --sims-per-step must divide --sims")
    aligned = (args.steps * K) % S == 0 and (args.warmup * K) % S == 0

    if args.rehearse:
        A = None
        ndev = world

        def synchronize():
            pass
    else:
        # libaz (and the /opt/rocm HIP runtime it is built for) is loaded before torch: torch
        # bundles its own libamdhip64.so.7 (same SONAME) and is only used here for the gloo
        # barrier / reduction between ranks -- the self-play path has no collective.
        import ctypes
        import azchess as A
        n = ctypes.c_int(0)
        A._lib.lib.az_device_count(ctypes.byref(n))
        ndev = n.value

        def synchronize():
            A._lib.check(A._lib.lib.az_device_synchronize(local))
    if args.same_device:
        local = 0
        ndev = max(ndev, world)
    if ndev < world or local >= ndev:
        raise SystemExit("bench.py: %d ranks need %d GPUs, %d visible" % (world, world, ndev))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    sh = shard(rank, world, G)

    def barrier():
        dist_barrier(world)
        synchronize()

    def phase(net, cache, steps, timing, G=G, S=S, K=K, warmup=None):
        """Self-play from startpos: warmup steps, then `steps` timed steps of K simulation steps; with
        `timing`, every 32nd simulation step carries HIP events (roofline / tree_walk), in the window
        or in a profile pass after it (persistent kernel).  G / S / K: the workload (default the
        headline's)."""
        warmup = args.warmup if warmup is None else warmup
        if args.rehearse:
            sp = RehearsalSelfPlay(G, S, sh["seed"])
        else:
            sp = A.SelfPlay(net, games=G, sims=S, device=local, continuous=True, seed=sh["seed"],
                            cache_capacity=cache)
        sp.reset()
        for _ in range(warmup):
            sp.run_sims(K)
            sp.drain()
        st0 = sp.search.stats()
        # the sampled steps (every 32nd) run as separate kernels bracketed by events: inside the
        # window when the engine steps with k_step + the tower (the events cost nothing measurable
        # there, and the roofline then times launches of the window itself); with the persistent
        # per-game kernel (C2) they would break it every 32 steps, so they go to a profile pass of
        # PROFILE_SIMS steps after the window
        persistent = bool(getattr(sp.search, "persistent", False))
        inwin = timing and not persistent
        sp.search.timing(reset=True, enable=inwin)
        barrier()
        t0 = time.perf_counter()
        finished = 0
        for _ in range(steps):
            f, _, _ = sp.run_sims(K)
            finished += f
            sp.drain()
        synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        st1 = sp.search.stats()
        digests = None
        if world > 1 and not args.rehearse:
            # per-rank fingerprint of the games (the roots' visit arrays at the end of the window):
            # distinct seeds must give distinct games on every rank
            import hashlib
            _, vis, dep = sp.search.read_roots()
            digests = [None] * world
            dist.all_gather_object(digests, hashlib.sha1(vis.tobytes() + dep.tobytes()).hexdigest()[:16])
        prof = min(PROFILE_SIMS, S) if timing and not inwin else 0
        if prof:
            sp.search.timing(reset=True, enable=True)
            sp.run_sims(prof)
            sp.drain()
            synchronize()
        tm = sp.search.timing(reset=False, enable=False)
        tm["persistent"] = persistent
        tm["profile_sim_steps"] = prof if prof else steps * K
        c = [st1[k] - st0[k] for k in ("sims", "evals", "terminal_leaves", "moves", "max_depth_sum", "cache_hits")]
        assert c[0] == G * K * steps, (c[0], G * K * steps)
        elapsed, tot = reduce_run(elapsed, c + [finished], world)
        del sp
        res = dict(zip(("sims", "evals", "terminal", "moves", "depth", "hits", "finished"), tot))
        res["rank_root_digests"] = digests
        return elapsed, res, tm, c[0]

    def roofline(tm, dtype, net, B=args.blocks, Fh=args.filters, G=G):
        """The fused tower over the timed region (HIP events around its launch on the engine stream,
        every 32nd simulation step).  achieved / frac = the MFMA FLOPs the kernel EXECUTES per launch
        (what the matrix pipe does: SURVEY 8d's roofline for the tower) / its measured time vs the
        dense peak of that MFMA dtype; with the Winograd tower that is 1/2.25 of the direct-conv
        multiplies on the residual convs.  algorithmic_tflops = the reference's direct-conv FLOPs
        (SURVEY 8a A6, 2*64*(171F + 18BF^2) per row) over the same time: an equivalent rate, not a
        fraction of any peak.  traffic = HBM bytes per launch from the committed PMC passes;
        traffic_ratio = traffic / the algorithmic bytes (every weight once + the rows' I/O)."""
        peak = PEAK_BF16_TFLOPS if dtype == "bf16" else PEAK_F32_TFLOPS
        launches = max(tm["conv_launches"], 1)
        rows = tm["conv_flop"] / max(tower_algo_flop_per_row(B, Fh), 1.0)
        secs = tm["conv_ms"] * 1e-3
        kname = net.tower_kernel if net is not None else "none (rehearsal)"
        wino = net is not None and net.winograd
        exec_row = tower_exec_flop_per_row(B, Fh, dtype, wino or net is None)
        exec_tflops = exec_row * rows / secs / 1e12 if secs > 0 else 0.0
        algo_tflops = tm["conv_flop"] / secs / 1e12 if secs > 0 else 0.0
        traffic, traffic_src = pmc_traffic(G, B, Fh, dtype, wino or net is None)
        # algorithmic bytes per launch: every weight of the net once (transformed Winograd weights
        # when the kernel uses them) + per row an 80-B packed position in and <= 218 priors out
        wb = 4.0 * ((16.0 if wino else 9.0) * Fh * Fh * 2 * B + 9 * 32 * Fh + 48 * Fh + 64 * 32 + 512 * 64) \
            if dtype != "bf16" else 2.0 * (9.0 * Fh * Fh * 2 * B + 9 * 32 * Fh) + 4.0 * (48 * Fh + 64 * 32 + 512 * 64)
        algo_bytes = wb + (rows / launches) * (80.0 + 218 * 4.0 + 4.0)
        return {"bound": "mfma", "achieved": exec_tflops, "peak": peak, "unit": "TFLOP/s",
                "frac": exec_tflops / peak, "traffic": traffic,
                "traffic_unit": "bytes/launch past L2 (PMC FETCH_SIZE x2 + WRITE_SIZE: L2-miss fabric requests, "
                                "Infinity-Cache hits included -- an upper bound on HBM bytes)",
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": algo_bytes,
                "traffic_ratio": (traffic / algo_bytes) if traffic else None,
                "kernel": "%s: input conv + %d residual convs + heads in one launch, %s; %d launches timed (HIP events "
                          "on every 32nd simulation step %s)"
                          % (kname, 2 * B, "v_mfma_f32_16x16x32_bf16" if dtype == "bf16" else "v_mfma_f32_16x16x4_f32",
                             tm["conv_launches"],
                             ("of a %d-step profile pass after the timed window" % tm["profile_sim_steps"])
                             if tm["persistent"] else "of the timed window"),
                "executed_flop_per_row": exec_row,
                "executed_note": ("Winograd F(2x2,3x3): the residual convs execute 1/2.25 of the direct-conv "
                                  "multiplies; input conv (19 planes in 12 packed k-steps) and the heads' MFMAs "
                                  "included"
                                  if wino else "direct convolution, input channels padded 19 -> 32, heads included"),
                "algorithmic_tflops": algo_tflops,
                "algorithmic_note": "direct-conv FLOPs of SURVEY 8a A6 (no heads) / tower time: an equivalent rate",
                "rows_per_launch": rows / launches,
                "avg_ms_per_launch": tm["conv_ms"] / launches}

    def make_net(dtype):
        if args.rehearse:
            return None
        return A.AlphaZero(args.blocks, args.filters, dtype=dtype, device=local, seed=42)

    # headline: reference precision, no FEN cache -> every non-terminal simulation evaluates its
    # leaf on the network
    legs = {}
    tl = time.perf_counter()
    net = make_net(args.dtype)
    elapsed, tot, tm, sims_rank = phase(net, 0, args.steps, True)
    legs["headline (incl. warmup, profile pass)"] = time.perf_counter() - tl
    roof = roofline(tm, args.dtype, net)
    del net
    sims_all, evals_all, term_all = tot["sims"], tot["evals"], tot["terminal"]
    fin_all, moves_all, depth_all = tot["finished"], tot["moves"], tot["depth"]

    # the bf16 throughput mode beside it (labelled; not the headline)
    bf16_res = None
    bf16_steps = args.steps if args.bf16_steps < 0 else args.bf16_steps
    if args.dtype == "f32" and bf16_steps > 0:
        tl = time.perf_counter()
        net16 = make_net("bf16")
        e16, t16, tm16, _ = phase(net16, 0, bf16_steps, True)
        bf16_res = {"value": t16["sims"] / e16, "unit": "sims/s", "steps": bf16_steps,
                    "ms_per_step": e16 / bf16_steps * 1e3, "dtype": "bf16",
                    "roofline": roofline(tm16, "bf16", net16),
                    "tolerance_vs_f32_oracle": TOLERANCE["bf16"],
                    "note": "bf16 weights/activations, f32 accumulate: narrower than the reference's f32, "
                            "reported beside the headline, not as it"}
        del net16
        legs["bf16_mode"] = time.perf_counter() - tl

    # C2 (BASELINE.json configs[1]) in steady state: 256 continuous games x 800 sims, 6x64 f32 net --
    # the persistent per-game kernel (one game per CU), its tower timed in a profile pass after
    # the window; beside games_per_hr_measured, which plays C2's games to the end
    c2_res = None
    if args.c2_steps > 0 and args.dtype == "f32":
        tl = time.perf_counter()
        net2 = None if args.rehearse else A.AlphaZero(6, 64, dtype="f32", device=local, seed=42)
        e2, t2, tm2, _ = phase(net2, 0, args.c2_steps, True, G=256, S=800, K=800, warmup=2)
        c2_res = {"value": t2["sims"] / e2, "unit": "sims/s", "n_gpus": world, "steps": args.c2_steps,
                  "sims_per_step": 800, "ms_per_step": e2 / args.c2_steps * 1e3, "dtype": "f32",
                  "config": "C2 (BASELINE.json configs[1]): 256 games/GPU x 800 sims/move, 6x64 f32 net, "
                            "continuous self-play from startpos (one move of every game per step)",
                  "evals_per_sim": t2["evals"] / max(t2["sims"], 1),
                  "roofline": roofline(tm2, "f32", net2, 6, 64, 256)}
        del net2
        legs["c2_steady"] = time.perf_counter() - tl

    # the reference's FEN cache (tree.rs:214-219) on the same window, on request
    cache_res = None
    if args.cache > 0:
        netc = make_net(args.dtype)
        e2, t2, _, _ = phase(netc, args.cache, args.steps, False)
        cache_res = {"value": t2["sims"] / e2, "unit": "sims/s", "evals_per_sim": t2["evals"] / max(t2["sims"], 1),
                     "cache_hit_frac": t2["hits"] / max(t2["sims"], 1), "entries": args.cache}
        del netc

    # measured games/hr: C2's configuration played to the end on every rank (training.rs:294-378)
    games_leg = None
    if args.games_leg and not args.rehearse:
        tl = time.perf_counter()
        games_leg = play_games_leg(A, local, sh["seed"], world, barrier, synchronize)
        legs["games_per_hr_measured (C2 played to the end)"] = time.perf_counter() - tl

    training = None
    if args.train_steps > 0 and not args.rehearse and not args.same_device:
        tl = time.perf_counter()
        training = train_phase(args, A, rank, world, local)
        legs["training"] = time.perf_counter() - tl
        tl = time.perf_counter()
        sh_train = train_phase(args, A, rank, world, local, mode="sharded")
        legs["training (sharded batch)"] = time.perf_counter() - tl
        if training is not None:
            training["sharded_batch"] = sh_train
    if rank != 0:
        dist.destroy_process_group()
        return
    value = sims_all / elapsed
    tower_tflops = tm["tower_flop"] / (tm["tower_ms"] * 1e-3) / 1e12 if tm["tower_ms"] > 0 else 0.0
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    # select_bytes covers every select walk of the timed window (or of the profile pass); the event
    # times cover its sampled launches (az_timing: every 32nd simulation step)
    sel_bytes_per_launch = tm["select_bytes"] / max(tm["profile_sim_steps"], 1)
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
        "data": ("rehearsal: CPU stub engine, no GPU -- exercises the rank plumbing only, the numbers measure nothing"
                 if args.rehearse else
                 "synthetic: random-init %dx%d weights (seed 42), self-play from startpos, Dirichlet noise on"
                 % (args.blocks, args.filters)),
        "config": {"workload": "%s: %d concurrent self-play games/GPU x %d sims/move, %d-block x %d-filter net"
                               % (config_name(G, S, args.blocks, args.filters), G, S, args.blocks, args.filters),
                   "games_per_gpu": G, "sims_per_move": S, "blocks": args.blocks, "filters": args.filters,
                   "sims_per_step": K,
                   "step": "%d simulation steps of every game (a move = %d steps)" % (K, S // K),
                   "window_move_aligned": aligned,
                   "fen_cache": "off (measured: 1 % hit rate over a 20-move C3 window, -14 % at C2; DESIGN.md section 6)",
                   "parallelism": ("games sharded %d-way, no collective (gloo barrier/max only)" % world) +
                                  (" -- TEST MODE: every rank on device 0 (--same-device), not a scaling "
                                   "measurement" if args.same_device else "")},
        "roofline": roof,
        "tower": {"algorithmic_tflops": tower_tflops,
                  "note": "the whole network's direct-conv FLOPs (SURVEY 8a A6, heads included) / tower time: an "
                          "equivalent rate, not a fraction of a peak (roofline.frac is the executed-MFMA fraction)",
                  "ms_per_sim_step": tm["tower_ms"] / max(tm["sim_steps"], 1),
                  "share_of_step": (tm["tower_ms"] / max(tm["sim_steps"], 1)) * K / (elapsed / args.steps * 1e3),
                  "share_note": "sampled launches (HIP events around every 32nd launch) x launches per step / wall time "
                                "per step; the event-bracketed launch starts on an idle pipe, so it can run ~0.5 % "
                                "longer than the average in-stream launch and this share can exceed 1 by that much "
                                "(roofline.achieved_wall_bound has no such bias)"},
        "tolerance_vs_f32_oracle": TOLERANCE[args.dtype],
        "bf16_mode": bf16_res,
        "tree_walk": {"kernel": "k_select", "achieved_gbs": sel_gbs, "peak_gbs": PEAK_HBM_GBS,
                      "frac": sel_gbs / PEAK_HBM_GBS,
                      # select_bytes counts every walk of the pass the events sample: the timed
                      # window, or the profile pass after it (persistent kernel)
                      "bytes_per_sim": tm["select_bytes"] / max(tm["profile_sim_steps"] * G, 1),
                      "avg_ms_per_launch": tm["select_ms"] / max(tm["select_launches"], 1)},
        "sim_step_ms": {k: tm[k + "_ms"] / max(tm["sim_steps"], 1)
                        for k in ("select", "expand", "encode", "tower", "heads", "backup")},
        "sim_kernels": ("k_sims32w<%d> for every simulation step of the window: one workgroup per game runs its backup, "
                        "select, expand and network evaluation with no grid-wide step boundary; the roofline / "
                        "tree_walk events come from a %d-step profile pass after the timed window, whose every-32nd "
                        "steps run as separate kernels" % (args.filters, tm["profile_sim_steps"])
                        ) if tm.get("persistent") else
                       "k_step (backup + select + expand) + the fused tower, two launches per simulation step",
        "evals_per_sim": evals_all / max(sims_all, 1),
        "terminal_leaf_frac": term_all / max(sims_all, 1),
        "with_fen_cache": cache_res,
        "avg_search_depth": depth_all / max(moves_all, 1),
        "games_finished_in_window": int(fin_all),
        # the games that happen to end inside a ~1-minute window of continuous self-play are not a
        # games/hr measurement: see games_per_hr_measured / _projected
        "games_per_hr": None,
        "games_per_hr_measured": games_leg,
        "c2_steady": c2_res,
        "rank_root_digests": tot["rank_root_digests"],
        "games_per_hr_projected": None,
        "cpu_baseline": None,
        "training": training,
    }
    gl_path = next((p for p in GAME_LENGTH if os.path.exists(p)), None)
    if (args.blocks, args.filters, S) == (20, 256, 800) and gl_path and not args.rehearse:
        with open(gl_path) as f:
            gl = json.load(f)
        # continuous self-play keeps every slot busy (a finished game restarts in its slot), so
        # the steady state plays sims/s / (sims/move * plies/game) games
        out["games_per_hr_projected"] = {
            "value": value * 3600.0 / (S * gl["plies_mean"]), "plies_per_game": gl["plies_mean"],
            "source": os.path.relpath(gl_path, ROOT), "game_length_net": gl.get("net"),
            "note": "projection, not a measurement: measured sims/s / (800 sims x mean plies of %d complete games "
                    "of a separate run); the timed window (%d x %d simulation steps) is too short for games to "
                    "finish" % (gl["games"], args.steps, K)}
    if roof and not args.rehearse and not tm.get("persistent") and elapsed > 0:
        # a bound free of the event bias: every launch of the window took at most wall / launches
        # (the tower is one of two launches per simulation step), so the executed rate is at least
        rpl = roof["rows_per_launch"]
        wb = roof["executed_flop_per_row"] * rpl * K * args.steps / elapsed / 1e12
        roof["achieved_wall_bound"] = wb
        roof["frac_wall_bound"] = wb / roof["peak"]
        roof["wall_bound_note"] = ("executed MFMA FLOPs of every tower launch of the timed window / the window's wall "
                                   "time (k_step, move completions and host work included): a strict lower bound "
                                   "on the tower's rate")
    if world == 1 and not args.no_cpu_baseline and not args.rehearse:
        tl = time.perf_counter()
        out["cpu_baseline"] = cpu_baseline(args.blocks, args.filters, args.cpu_threads, args.cpu_games,
                                           args.cpu_sims)
        legs["cpu_baseline"] = time.perf_counter() - tl
        # SURVEY 8d asks for the host's cores: beside the box's 16-thread CPU share, the same sample at
        # one GPU's share of the host (nproc / 8 on an 8-GPU node)
        share = max(1, len(os.sched_getaffinity(0)) // 8)
        if share != args.cpu_threads:
            tl = time.perf_counter()
            cb = cpu_baseline(args.blocks, args.filters, share, args.cpu_games, args.cpu_sims, port=False)
            out["cpu_baseline"]["per_gpu_share"] = {k: cb[k] for k in ("value", "unit", "threads", "sample")}
            q = cgroup_cpus()
            out["cpu_baseline"]["per_gpu_share"]["note"] = (
                "nproc / 8 threads: one GPU's share of an 8-GPU host" +
                ("; this process's cgroup allows %.0f CPUs, so %d threads oversubscribe it (the 16-thread value "
                 "above is the box's own share)" % (q, share) if q and q < share else ""))
            legs["cpu_baseline (per-GPU share)"] = time.perf_counter() - tl
    out["legs_wall_s"] = {k: round(v, 2) for k, v in legs.items()}
    out["legs_note"] = "wall time of every leg this run executed (rank 0); only the headline's timed window is `value`"
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())

"""N>1 path on CPU: world_size-2 gloo processes run the sharding / barrier / reduction logic
bench.py uses (no GPU; the self-play path itself has no collective)."""
import os
import socket



def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "alphazero-chess_amd"))
    import torch.distributed as dist
    from azchess.dist import barrier, reduce_run, shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = shard(rank, world, 2048)
    barrier(world)
    elapsed = 1.0 + rank                      # rank 1 is the slowest
    sims = 2048 * 800 * 3
    t, tot = reduce_run(elapsed, [sims, sims - rank, rank], world)
    q.put((rank, sh["seed"], sh["first_game"], t, tot))
    dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_reduction():
    import torch.multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = {r[1] for r in res}
    assert len(seeds) == world                       # distinct game streams per rank
    assert [r[2] for r in res] == [0, 2048]
    for r in res:
        assert r[3] == 2.0                           # max over ranks
        assert r[4] == [2 * 2048 * 800 * 3, 2 * 2048 * 800 * 3 - 1, 1]


def _bench(args, env=None, timeout=240):
    import json
    import subprocess
    import sys
    from conftest import ROOT
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=timeout, env=e)
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    return out.returncode, [json.loads(l) for l in lines], out.stderr


def test_bench_gpus_flag_spawns_the_ranks():
    """`bench.py --gpus 2` with no torchrun environment starts 2 ranks itself (the same code path
    a GPU run takes, with the CPU stub engine): one JSON line from rank 0, n_gpus = 2, value =
    the simulations of BOTH ranks / the max-over-ranks time."""
    G, K, steps = 64, 8, 3
    rc, lines, err = _bench(["--gpus", "2", "--rehearse", "--steps", str(steps), "--warmup", "1", "--games", str(G),
                             "--sims", "16", "--sims-per-step", str(K), "--bf16-steps", "0"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 2 and r["steps"] == steps and r["scaling"] == "weak"
    sims = r["value"] * r["ms_per_step"] * 1e-3 * steps
    assert abs(sims - 2 * G * K * steps) < 1e-6 * sims
    assert "2-way" in r["config"]["parallelism"]


def test_bench_eight_ranks_c4_layout():
    """configs[3] (C4: games sharded 8-way, no collective on the path) rehearsed on the CPU: `bench.py
    --gpus 8` spawns 8 ranks over gloo with the stub engine (the driver's 8-GPU scaling run takes the
    same code path with the real engine, one rank per GPU): one JSON line from rank 0, n_gpus = 8,
    value = the simulations of all 8 ranks / the max-over-ranks time, 8 distinct game seeds."""
    G, K, steps = 32, 8, 2
    rc, lines, err = _bench(["--gpus", "8", "--rehearse", "--steps", str(steps), "--warmup", "1", "--games", str(G),
                             "--sims", "16", "--sims-per-step", str(K), "--bf16-steps", "0", "--c2-steps", "0",
                             "--games-leg", "0", "--train-steps", "0"], timeout=600)
    assert rc == 0, err[-2000:]
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 8 and r["scaling"] == "weak" and "8-way" in r["config"]["parallelism"]
    sims = r["value"] * r["ms_per_step"] * 1e-3 * steps
    assert abs(sims - 8 * G * K * steps) < 1e-6 * sims


def test_bench_rejects_world_mismatch():
    rc, lines, err = _bench(["--gpus", "1", "--rehearse", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert rc != 0 and not lines and "WORLD_SIZE=2" in err


# ------------------------------------------------------------ one replay buffer over the ranks
def _rank_steps(rank, n=120):
    """Synthetic drained EpisodeSteps of one rank: random playouts of <= 8 plies from the startpos
    (so the two ranks reach many of the same positions: cross-rank merges), random visit counts on
    the legal indices, one record with no visits and one with the maximum 224."""
    import numpy as np
    import azchess as A
    from azchess import _lib as L
    rng = np.random.default_rng(1000 + rank)
    out = []
    for i in range(n):
        gs = A.GameState()
        for _ in range(int(rng.integers(0, 9))):
            idx = gs.position.legal_indices()
            if len(idx) == 0 or int(A.play_move(gs, int(rng.choice(idx)))) != 0:
                break
        st = L.AzEpisodeStep()
        st.game_id, st.ply, st.action, st.search_depth = rank * 1000 + i, i, 0, 3
        st.final_value = float(np.float32(rng.uniform(-1, 1)))
        st.state = gs.position._p
        idx = np.unique(gs.position.legal_indices())
        nv = 0 if i == 7 else len(idx)
        st.nvis = nv
        for k in range(nv):
            st.vis_idx[k], st.vis_n[k] = int(idx[k]), int(rng.integers(1, 40))
        if i == 11:                                   # the record's full capacity
            st.nvis = 224
            for k in range(224):
                st.vis_idx[k], st.vis_n[k] = k, k + 1
        out.append(st)
    return out


def _replay_worker(rank, world, port, path, q):
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "alphazero-chess_amd"))
    import azchess  # noqa: F401  (before torch: binds libaz to /opt/rocm's HIP runtime)
    import torch.distributed as dist
    from azchess.dist import allgather_bytes
    from azchess.memory import ReplayBuffer, add_from_ranks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = ReplayBuffer(capacity=150)                 # small: FIFO eviction happens on the union
    new, added = add_from_ranks(buf, _rank_steps(rank), allgather_bytes)
    buf.save(path + "_%d" % rank)
    q.put((rank, new, added, len(buf)))
    dist.destroy_process_group()


def test_two_rank_gloo_shared_replay_is_one_buffer(tmp_path):
    """every rank's drained EpisodeSteps go to every rank in (rank, drain)
    order (memory.add_from_ranks over azchess.dist.allgather_bytes, gloo), so the two ranks'
    replicas save byte-identical files, equal to ONE buffer fed the concatenation in rank order --
    the reference's single memory.rs buffer (memory.rs:41-96) with its FEN dedup / running means and
    FIFO eviction over the union."""
    import torch.multiprocessing as mp
    from azchess.memory import ReplayBuffer
    world, port = 2, _free_port()
    path = str(tmp_path / "replay")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_replay_worker, args=(r, world, port, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    one = ReplayBuffer(capacity=150)
    new = one.add_many(_rank_steps(0) + _rank_steps(1))
    one.save(path + "_one")
    raw = [open(path + s, "rb").read() for s in ("_0", "_1", "_one")]
    assert raw[0] == raw[1] == raw[2]
    assert [r[1] for r in res] == [new, new] and [r[2] for r in res] == [240, 240]
    assert res[0][3] == len(one) == 150 and new > 150          # evictions happened
    assert new < 240                                            # and merges


def test_pack_unpack_steps_round_trip():
    import ctypes
    import numpy as np
    from azchess import _lib as L
    from azchess.memory import pack_steps, unpack_steps
    steps = _rank_steps(0, 20)
    back = unpack_steps(pack_steps(steps))
    assert len(back) == 20
    for a, b in zip(steps, back):
        na = np.frombuffer(ctypes.string_at(ctypes.addressof(a), ctypes.sizeof(a)), np.uint8)
        nb = np.frombuffer(ctypes.string_at(ctypes.addressof(b), ctypes.sizeof(b)), np.uint8)
        nv = a.nvis
        assert np.array_equal(na[:112], nb[:112])               # header, position (padding included)
        assert list(a.vis_idx[:nv]) == list(b.vis_idx[:nv]) and list(a.vis_n[:nv]) == list(b.vis_n[:nv])
        assert not any(b.vis_idx[nv:]) and not any(b.vis_n[nv:])
    assert len(unpack_steps(pack_steps([]))) == 0
    bad = L.AzEpisodeStep()
    bad.nvis = 225
    try:
        pack_steps([bad])
        assert False, "nvis 225 packed"
    except ValueError:
        pass
    try:
        unpack_steps(pack_steps(steps)[:-2])
        assert False, "truncated payload accepted"
    except ValueError:
        pass


def test_train_world2_argument_checks_before_any_device_call():
    """train() at world > 1 (the reference's train(): one shared buffer, sharded batch) refuses on
    the host, before a trainer touches a GPU: a global batch smaller than the world, and a shared
    buffer with no way to exchange EpisodeSteps (no allgather and no torch.distributed group)."""
    import pytest
    import azchess as A
    red = (lambda buf: None, 0, 2)
    with pytest.raises(ValueError, match="smaller than world"):
        A.train(1, reducer=red, batch_size=1, allgather=lambda b: [b, b])
    with pytest.raises(ValueError, match="allgather"):
        A.train(1, reducer=red)
    with pytest.raises(ValueError, match="not both"):
        A.train(1, reducer=red, comm=(b"", 0, 2))

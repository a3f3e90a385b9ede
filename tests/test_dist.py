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


def test_bench_rejects_world_mismatch():
    rc, lines, err = _bench(["--gpus", "1", "--rehearse", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert rc != 0 and not lines and "WORLD_SIZE=2" in err

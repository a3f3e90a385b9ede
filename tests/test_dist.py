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

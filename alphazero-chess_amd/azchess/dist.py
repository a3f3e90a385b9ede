"""Multi-GPU self-play sharding: one process per GPU, games are independent, so
the only communication is a barrier around the timed region and one reduction of the
counters at the end -- no collective on the search / inference path."""
import os

SEED_STRIDE = 1000003


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(rank, world, games_per_rank, base_seed=42):
    """Game slots and RNG stream of one rank: distinct seeds => distinct games."""
    assert 0 <= rank < world
    return {"device": None, "games": games_per_rank, "seed": base_seed + SEED_STRIDE * rank,
            "first_game": rank * games_per_rank}


def reduce_run(elapsed, counters, world, device=None):
    """Max over ranks of the elapsed time, sum over ranks of the counters."""
    if world == 1:
        return elapsed, list(counters)
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(v) for v in counters], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [float(v) for v in c.tolist()]


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()

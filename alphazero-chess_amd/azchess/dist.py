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


def allgather_bytes(payload, group=None):
    """Every rank's byte string, in rank order, over the initialised torch.distributed group (gloo:
    host tensors; nccl: tensors on the current device).  Used once per self-play pass to replicate
    the replay buffer (memory.add_from_ranks), never on the search path."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = torch.device("cpu")
    if dist.get_backend(group) != "gloo":
        dev = torch.device("cuda", torch.cuda.current_device())
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(max(sizes), 1)
    buf = torch.zeros(m, dtype=torch.uint8, device=dev)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    outs = [torch.empty(m, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return [o[:s].cpu().numpy().tobytes() for o, s in zip(outs, sizes)]


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()

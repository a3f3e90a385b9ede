"""The sharded-batch training step (az_trainer_set_sharded) across two real
PROCESSES on one GPU: each rank is its own process with its own trainer, the exchange runs over
torch.distributed gloo through az_trainer_set_host_reducer (RCCL refuses two ranks on one device;
the driver's 8-GPU run takes the RCCL path).  Checks, after two steps on the two shards of one
global batch: both ranks hold bit-identical parameters, and they equal the in-process two-trainer
run with a host reducer that adds rank 0's buffer to rank 1's (gloo's two-rank sum is that same
float32 addition), so process isolation, the gloo exchange and the per-rank shard slicing change
nothing."""
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

import azchess as A

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOCKS, FILTERS, GB, STEPS = 2, 256, 96, 2

_RANK = r"""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.environ["AZ_ROOT"], "alphazero-chess_amd"))
import azchess as A
import torch
import torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
d = np.load(os.environ["AZ_BATCH"])
n = d["planes"].shape[0] // world
sl = slice(rank * n, (rank + 1) * n)
tr = A.Trainer(%d, %d, weights=d["w"], max_batch=n)
def reduce(buf):
    t = torch.from_numpy(buf.copy())
    dist.all_reduce(t)
    buf[:] = t.numpy()
tr.set_host_reducer(reduce, rank, world)
tr.set_sharded(True)
losses = [tr.step(d["planes"][sl], d["pol"][sl], d["val"][sl], A.get_cyclical_lr(it)) for it in range(%d)]
np.save(os.environ["AZ_OUT"] + "_%%d.npy" %% rank, tr.params())
print(json.dumps({"rank": rank, "losses": [list(map(float, l)) for l in losses]}))
dist.destroy_process_group()
""" % (BLOCKS, FILTERS, STEPS)


def _batch():
    rng = np.random.default_rng(77)
    planes = (rng.random((GB, 19, 64)) < 0.1).astype(np.float32)
    pol = rng.random((GB, 4096)).astype(np.float32)
    pol /= pol.sum(1, keepdims=True)
    val = rng.uniform(-1, 1, GB).astype(np.float32)
    return planes, pol, val


def test_sharded_step_two_processes_gloo_matches_in_process(require_gpu, tmp_path):
    w = A.random_weights(BLOCKS, FILTERS, seed=31)
    planes, pol, val = _batch()
    bpath = str(tmp_path / "batch.npz")
    np.savez(bpath, w=w, planes=planes, pol=pol, val=val)
    out = str(tmp_path / "params")
    port = 29500 + os.getpid() % 1000
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   AZ_ROOT=ROOT, AZ_BATCH=bpath, AZ_OUT=out)
        procs.append(subprocess.Popen([sys.executable, "-c", _RANK], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    res = []
    try:
        for p in procs:
            so, se = p.communicate(timeout=240)
            assert p.returncode == 0, se[-3000:]
            res.append(json.loads([l for l in so.splitlines() if l.startswith("{")][-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    p0, p1 = np.load(out + "_0.npy"), np.load(out + "_1.npy")
    assert np.array_equal(p0, p1)
    assert res[0]["losses"] == res[1]["losses"]

    # the same two shards as two trainers in this process, rank 0's buffer + rank 1's
    n = GB // 2
    slots, bar = [None, None], threading.Barrier(2, timeout=60)

    def reducer(rank):
        def reduce(buf):
            slots[rank] = buf.copy()
            bar.wait()
            buf[:] = slots[0] + slots[1]
            bar.wait()
        return reduce

    params, losses, errs = [None, None], [None, None], []

    def run(rank):
        try:
            sl = slice(rank * n, (rank + 1) * n)
            tr = A.Trainer(BLOCKS, FILTERS, weights=w, max_batch=n)
            tr.set_host_reducer(reducer(rank), rank, 2)
            tr.set_sharded(True)
            losses[rank] = [list(map(float, tr.step(planes[sl], pol[sl], val[sl], A.get_cyclical_lr(it))))
                            for it in range(STEPS)]
            params[rank] = tr.params()
        except Exception as e:      # surfaced below
            errs.append(e)
    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not errs, errs
    assert np.array_equal(params[0], p0), np.abs(params[0] - p0).max()
    assert losses[0] == res[0]["losses"]


_TRAIN_RANK = r"""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.environ["AZ_ROOT"], "alphazero-chess_amd"))
import azchess as A
import torch
import torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
def reduce(buf):
    t = torch.from_numpy(buf.copy())
    dist.all_reduce(t)
    buf[:] = t.numpy()
batches = []
tr, rep, hist = A.train(1, blocks=2, filters=64, games=8, sims=4, min_replay=48, train_steps=2, batch_size=32,
                        seed=9, reducer=(reduce, rank, world),
                        log_batch=lambda it, b, pl, po, va, lo, hi: batches.append((pl.sum(), lo, hi)))
out = os.environ["AZ_OUT"] + "_%d" % rank
np.save(out + ".npy", tr.params())
rep.save(out + ".replay")
print(json.dumps({"rank": rank, "hist": {k: v for k, v in hist[0].items() if isinstance(v, (int, float, bool))},
                  "batches": [[float(s), lo, hi] for s, lo, hi in batches]}))
dist.destroy_process_group()
"""


def test_train_two_processes_one_global_buffer(require_gpu, tmp_path):
    """train() at world 2 as two real processes on one GPU, with its defaults: the EpisodeSteps
    exchanged by azchess.dist.allgather_bytes over torch.distributed gloo (the production path of
    DESIGN 7.1), the sharded step's exchanges through a gloo host reducer.  Both processes end with
    byte-identical replay buffers and bit-identical parameters, drew the same global batch each step
    and trained its two halves."""
    out = str(tmp_path / "rank")
    port = 29700 + os.getpid() % 1000
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   AZ_ROOT=ROOT, AZ_OUT=out)
        procs.append(subprocess.Popen([sys.executable, "-c", _TRAIN_RANK], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    res = []
    try:
        for p in procs:
            so, se = p.communicate(timeout=240)
            assert p.returncode == 0, se[-3000:]
            res.append(json.loads([l for l in so.splitlines() if l.startswith("{")][-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert np.array_equal(np.load(out + "_0.npy"), np.load(out + "_1.npy"))
    assert open(out + "_0.replay", "rb").read() == open(out + "_1.replay", "rb").read()
    h0, h1 = res[0]["hist"], res[1]["hist"]
    assert h0["shared_replay"] and h0["shard_batch"] and h0["replay"] == h1["replay"] >= 48
    assert h0["episode_steps_global"] == h0["episode_steps"] + h1["episode_steps"]
    assert h0["policy_loss"] == h1["policy_loss"]
    b0, b1 = res[0]["batches"], res[1]["batches"]
    assert [b[0] for b in b0] == [b[0] for b in b1]               # the same global batch
    assert all(b[1:] == [0, 16] for b in b0) and all(b[1:] == [16, 32] for b in b1)

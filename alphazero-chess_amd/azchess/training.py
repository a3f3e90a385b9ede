"""training.rs mirror of the self-play hot path: EpisodeStep, run_episode,
run_all_episodes and process_batch (src/training.rs:15-38, 294-422).

The reference runs one tokio task per game and batches leaf evaluations through an
mpsc channel; here all games of a GPU advance in lockstep inside libaz and every
simulation step evaluates all pending leaves in one batch, with nothing crossing PCIe
until a move's EpisodeSteps are drained.
"""
import ctypes as C
import time
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .chess import Position, to_tensor
from .parameters import (BATCH_SIZE, MIN_REPLAY_SIZE, NUM_EPISODES, NUM_FILTERS, NUM_RES_BLOCKS, NUM_SIMULATIONS,
                         NUM_TRAIN_STEPS, SEED)
from .tree import BatchedSearch


@dataclass
class EpisodeStep:                   # training.rs:15-20
    state: Position
    improved_policy: np.ndarray      # [4096] = visits / sum(visits)
    final_value: float
    search_depth: int
    game_id: int = 0
    ply: int = 0
    action: int = 0
    result: int = 0
    visits: dict = None


def _convert(st):
    pos = Position(L.AzPos.from_buffer_copy(st.state))
    n = st.nvis
    idx = np.frombuffer(st.vis_idx, np.uint16)[:n].astype(np.int64)
    cnt = np.frombuffer(st.vis_n, np.uint16)[:n].astype(np.float32)
    pol = np.zeros(4096, np.float32)
    tot = np.float32(cnt.sum())
    pol[idx] = cnt / tot
    return EpisodeStep(pos, pol, float(st.final_value), int(st.search_depth), int(st.game_id), int(st.ply),
                       int(st.action), int(st.result), {int(i): int(c) for i, c in zip(idx, cnt) if c})


class SelfPlay:
    """run_all_episodes engine: G game slots on one GPU."""

    def __init__(self, model=None, games=100, device=0, continuous=False, **cfg):
        self.search = BatchedSearch(model, games=games, device=device, continuous=continuous, **cfg)
        self.games = games

    def reset(self):
        self.search.check(L.lib.az_selfplay_reset(self.search._h))

    def step(self):
        fin, act = C.c_int(), C.c_int()
        self.search.check(L.lib.az_selfplay_step(self.search._h, C.byref(fin), C.byref(act)))
        return fin.value, act.value

    def run_sims(self, nsims):
        """The next `nsims` simulation steps of the current move of every game; when the move
        completes, its action choice / play / re-root follow as in step().  Returns
        (finished, active, move_done); active is -1 while the move is in progress."""
        fin, act, done = C.c_int(), C.c_int(), C.c_int()
        self.search.check(L.lib.az_selfplay_run_sims(self.search._h, int(nsims), C.byref(fin), C.byref(act), C.byref(done)))
        return fin.value, act.value, bool(done.value)

    def drain(self):
        return [_convert(s) for s in self.drain_raw()]

    _drain_buf = None

    def drain_raw(self):
        """EpisodeSteps of the games that ended, as the engine's az_episode_step records (what
        ReplayBuffer.add takes directly): a right-sized array per call (the 4 MB staging buffer is
        reused, so a pass that keeps its drains holds only the steps themselves)."""
        if self._drain_buf is None:
            self._drain_buf = (L.AzEpisodeStep * 4096)()
        buf, parts = self._drain_buf, []
        while True:
            n = L.check(L.lib.az_selfplay_drain(self.search._h, buf, 4096))
            if n:
                arr = (L.AzEpisodeStep * n)()
                C.memmove(arr, buf, n * C.sizeof(L.AzEpisodeStep))
                parts.append(arr)
            if n < 4096:
                break
        if len(parts) == 1:
            return parts[0]
        return (L.AzEpisodeStep * sum(len(p) for p in parts))(*[s for p in parts for s in p])


def run_all_episodes(model=None, games=100, max_moves=1000, device=0, **cfg):
    """training.rs:340-378: play `games` games from startpos to the end; returns
    (avg_batch_size, steps) like the reference (steps of all games, game order)."""
    sp = SelfPlay(model, games=games, device=device, continuous=False, **cfg)
    sp.reset()
    steps = []
    for _ in range(max_moves):
        _, active = sp.step()
        steps += sp.drain()
        if active == 0:
            break
    st = sp.search.stats()
    sims = max(st["sims"], 1)
    avg_batch = st["evals"] / max(sims / games, 1)
    return avg_batch, steps


def run_episode(model=None, device=0, **cfg):
    """training.rs:294-338 for a single game."""
    return run_all_episodes(model, games=1, device=device, **cfg)[1]


def process_batch(states, model):
    """training.rs:380-422: one batched forward over the requests' positions."""
    x = np.concatenate([to_tensor(s) for s in states], 0)
    return model.forward(x)


# ---------------------------------------------------------------- train()
def get_cyclical_lr(iteration):
    """training.rs:424-441"""
    return float(L.lib.az_cyclical_lr(int(iteration)))


def comm_unique_id():
    """RCCL unique id (128 bytes) for Trainer.set_comm; create on rank 0, share over the host."""
    buf = (C.c_char * 128)()
    L.check(L.lib.az_comm_unique_id(buf, 128))
    return bytes(buf)


class Trainer:
    """The reference's training half of train() (training.rs:137-190) on one GPU: the model's
    flat parameters, the AdamW state (training.rs:63-66) and every activation of a batch live
    in HBM; one step = forward in training mode + compute_gradients + optimizer.step.
    Data-parallel over RCCL with set_comm (gradients summed over ranks before clipping)."""

    def __init__(self, blocks, filters, weights=None, max_batch=512, device=0, seed=42):
        from .agent import random_weights
        if weights is None:
            weights = random_weights(blocks, filters, seed)
        self.blocks, self.filters, self.device = blocks, filters, device
        self.n = int(L.lib.az_net_num_params(blocks, filters))
        w = np.ascontiguousarray(weights, np.float32)
        h = C.c_void_p()
        L.check(L.lib.az_trainer_create(blocks, filters, L.fptr(w), w.size, max_batch, device, C.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            L.lib.az_trainer_destroy(h)
            self._h = None

    @staticmethod
    def _batch(planes, tpol, tval):
        planes = np.ascontiguousarray(planes, np.float32).reshape(-1, 19 * 64)
        tpol = np.ascontiguousarray(tpol, np.float32).reshape(-1, 4096)
        tval = np.ascontiguousarray(tval, np.float32).reshape(-1)
        assert planes.shape[0] == tpol.shape[0] == tval.shape[0]
        return planes, tpol, tval

    def compute_gradients(self, planes, tpol, tval):
        planes, tpol, tval = self._batch(planes, tpol, tval)
        loss = np.zeros(2, np.float32)
        self._check(L.lib.az_trainer_compute_grads(self._h, L.fptr(planes), L.fptr(tpol), L.fptr(tval),
                                                   planes.shape[0], L.fptr(loss)))
        return float(loss[0]), float(loss[1])

    def apply(self, lr):
        self._check(L.lib.az_trainer_apply(self._h, float(lr)))

    def step(self, planes, tpol, tval, lr):
        planes, tpol, tval = self._batch(planes, tpol, tval)
        loss = np.zeros(2, np.float32)
        self._check(L.lib.az_trainer_step(self._h, L.fptr(planes), L.fptr(tpol), L.fptr(tval), planes.shape[0],
                                          float(lr), L.fptr(loss)))
        return float(loss[0]), float(loss[1])

    def params(self):
        out = np.empty(self.n, np.float32)
        L.check(L.lib.az_trainer_get_params(self._h, L.fptr(out), self.n))
        return out

    def grads(self):
        out = np.empty(self.n, np.float32)
        L.check(L.lib.az_trainer_get_grads(self._h, L.fptr(out), self.n))
        return out

    def relu_masks(self, batch):
        """ReLU masks of the last forward in forward order (parity tests): tower layers as
        NCHW [B, F, 8, 8], heads [B, 40, 8, 8], value hidden [B, 64]."""
        out, F = [], self.filters
        for layer in range(2 * self.blocks + 3):
            if layer <= 2 * self.blocks:
                a = np.empty(batch * 64 * F, np.float32)
            elif layer == 2 * self.blocks + 1:
                a = np.empty(batch * 64 * 64, np.float32)
            else:
                a = np.empty(batch * 64, np.float32)
            L.check(L.lib.az_trainer_relu_output(self._h, layer, L.fptr(a), a.size))
            if layer <= 2 * self.blocks:
                out.append(a.reshape(batch, 8, 8, F).transpose(0, 3, 1, 2) > 0)
            elif layer == 2 * self.blocks + 1:
                out.append(a.reshape(batch, 8, 8, 64).transpose(0, 3, 1, 2)[:, :40] > 0)
            else:
                out.append(a.reshape(batch, 64) > 0)
        return out

    _pending = None

    def _check(self, rc):
        """L.check for calls that may run the host reducer: a KeyboardInterrupt / SystemExit raised
        inside it is re-raised here, after the C call has returned its error."""
        e = self._pending[0] if self._pending else None
        if e is not None:
            self._pending[0] = None
            raise e
        return L.check(rc)

    def set_comm(self, unique_id, rank, world):
        buf = (C.c_char * 128).from_buffer_copy(unique_id)
        L.check(L.lib.az_trainer_set_comm(self._h, buf, int(rank), int(world)))

    def set_host_reducer(self, reduce, rank, world):
        """Data-parallel steps with the exchange done on the host: reduce(buf) must replace the
        float32 array buf by its element-wise sum over the `world` ranks (in place).  An exception
        inside it fails the step."""
        def fn(_ctx, ptr, n):
            try:
                reduce(np.ctypeslib.as_array(ptr, shape=(n,)))
                return 0
            except BaseException as e:       # nothing may unwind through the C frames; a
                import traceback             # KeyboardInterrupt / SystemExit is re-raised by
                traceback.print_exc()        # _check once the C call has returned (as tree.py)
                if not isinstance(e, Exception):
                    self._pending[0] = e
                return 1
        self._pending = [None]
        self._reduce_fn = L.ALLREDUCE_FN(fn)   # kept alive with the trainer
        L.check(L.lib.az_trainer_set_host_reducer(self._h, C.cast(self._reduce_fn, C.c_void_p), None, int(rank),
                                                  int(world)))

    def set_sharded(self, on=True):
        """Sharded batch (az_trainer_set_sharded): this rank's batches are its shard of one global
        batch -- the reference's single 512 step (training.rs:137-159) split over the ranks, with
        BatchNorm statistics, the BN backward and the loss over the whole global batch."""
        L.check(L.lib.az_trainer_set_sharded(self._h, int(bool(on))))

    def timing(self, reset=False):
        """(step_ms, allreduce_ms, steps): device time summed over the steps since the last reset."""
        a, b, n = C.c_double(), C.c_double(), C.c_int64()
        L.check(L.lib.az_trainer_timing(self._h, C.byref(a), C.byref(b), C.byref(n), int(reset)))
        return a.value, b.value, n.value

    def time_exchanges(self, on=True):
        """HIP events around every exchange of the following steps (for exchange_stats' time)."""
        L.check(L.lib.az_trainer_time_exchanges(self._h, int(bool(on))))

    def exchange_stats(self, reset=False):
        """(collectives, steps, exchange_ms): the data-parallel exchanges since the last reset --
        how many, over how many applied steps, and (while time_exchanges is on) their device time."""
        a, b, c = C.c_int64(), C.c_int64(), C.c_double()
        L.check(L.lib.az_trainer_exchange_stats(self._h, C.byref(a), C.byref(b), C.byref(c), int(reset)))
        return a.value, b.value, c.value

    def model(self, dtype="f32"):
        """model.valid() for self-play (training.rs:83): an inference net with the current weights,
        f32 like the reference's Cuda<f32> backend (bf16 is an explicit throughput opt-in)."""
        from .agent import AlphaZero
        return AlphaZero(self.blocks, self.filters, weights=self.params(), dtype=dtype, device=self.device)


def sample_seed(seed, iteration, step, rank=None):
    """Seed of one training step's replay sample.  rank None: the seed every rank shares (one global
    batch drawn from the replicated buffer); else a per-rank stream."""
    s = (seed << 20) ^ (iteration << 8) ^ step
    return s if rank is None else s ^ rank << 40


def shard_bounds(n, rank, world):
    """This rank's contiguous rows [lo, hi) of an n-row global batch."""
    return rank * n // world, (rank + 1) * n // world


def _default_allgather():
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        raise ValueError("train: world > 1 with a shared replay buffer needs allgather= or an initialised "
                         "torch.distributed group")
    from .dist import allgather_bytes
    return allgather_bytes


def train(iterations, blocks=NUM_RES_BLOCKS, filters=NUM_FILTERS, games=NUM_EPISODES, sims=NUM_SIMULATIONS,
          min_replay=MIN_REPLAY_SIZE, train_steps=NUM_TRAIN_STEPS, batch_size=BATCH_SIZE, replay=None, trainer=None,
          device=0, seed=SEED, dtype="f32", comm=None, shard_batch=None, reducer=None, shared_replay=None,
          allgather=None, log=None, log_batch=None):
    """train() (training.rs:39-275) without the TUI, arena and Elo (SKIP_VALIDATION = true,
    parameters.rs:35): per iteration, self-play `games` games with model.valid() until the replay
    buffer holds min_replay unique positions, then train_steps AdamW steps on batches of
    batch_size at get_cyclical_lr(iteration); the new model replaces the old one.

    Data parallel (comm = (unique_id, rank, world) over RCCL, or reducer = (reduce, rank, world)
    through a host callback, Trainer.set_host_reducer): every rank plays its own games (seed offset
    by rank), and by default (world > 1) the loop computes the reference's train() itself:
      * shared_replay (default on): ONE replay buffer (memory.rs:41-96), replicated -- after each
        self-play pass the ranks exchange their drained EpisodeSteps through allgather(bytes) ->
        [bytes per rank] (default: azchess.dist.allgather_bytes over torch.distributed) and every
        rank adds the union in (rank, drain) order (memory.add_from_ranks), so MIN_REPLAY_SIZE is
        tested on the global length and every rank leaves self-play together;
      * shard_batch (default on): each step is the reference's ONE batch of batch_size
        (training.rs:137-138), drawn with a seed shared by all ranks, and each rank trains its
        contiguous slice (az_trainer_set_sharded: BatchNorm statistics, BN backward and the loss
        over the whole batch).
    Labelled opt-ins: shard_batch=False trains batch_size per rank (global batch batch_size x world,
    per-rank BatchNorm, averaged gradients); shared_replay=False keeps one buffer per rank.
    log_batch(iteration, step, planes, policy, value, lo, hi): each step's drawn batch and this
    rank's rows of it.  Returns (trainer, replay, per-iteration stats)."""
    from .memory import ReplayBuffer, add_from_ranks
    if comm and reducer:
        raise ValueError("train: comm (RCCL) or reducer (host), not both")
    rank, world = (comm[1], comm[2]) if comm else (reducer[1], reducer[2]) if reducer else (0, 1)
    shard_batch = world > 1 if shard_batch is None else bool(shard_batch)
    shared_replay = world > 1 if shared_replay is None else bool(shared_replay)
    if shard_batch and batch_size < world:
        raise ValueError("shard_batch: batch_size %d is smaller than world %d" % (batch_size, world))
    if shared_replay and world > 1 and allgather is None:
        allgather = _default_allgather()
    # the largest shard a rank can get of a (possibly short) global batch
    local_batch = -(-batch_size // world) if shard_batch else batch_size
    if trainer is None:
        trainer = Trainer(blocks, filters, max_batch=local_batch, device=device, seed=seed)
        if comm:
            trainer.set_comm(*comm)
        elif reducer:
            trainer.set_host_reducer(*reducer)
    trainer.set_sharded(shard_batch)   # a caller's trainer too (its comm / reducer is the caller's)
    replay = replay if replay is not None else ReplayBuffer()
    history = []
    for iteration in range(iterations):
        t0 = time.perf_counter()
        model = trainer.model(dtype)
        new_unique, plays, sims_done, games_done, steps_done, moves_done, finished = 0, 0, 0, 0, 0, 0, 0
        steps_global = 0
        while True:
            sp = SelfPlay(model, games=games, sims=sims, device=device, continuous=False,
                          seed=seed + 1000003 * rank + 7919 * iteration + 104729 * plays)
            sp.reset()
            local = []
            while True:
                _, active = sp.step()
                drained = sp.drain_raw()
                steps_done += len(drained)
                if shared_replay and world > 1:
                    local.append(drained)
                else:
                    new_unique += replay.add_many(drained)
                if active == 0:
                    break
            if shared_replay and world > 1:
                nsteps = sum(len(d) for d in local)
                allsteps = (L.AzEpisodeStep * nsteps)()
                o = 0
                for d in local:   # this pass's drains in order, one contiguous array
                    C.memmove(C.byref(allsteps, o * C.sizeof(L.AzEpisodeStep)), d, len(d) * C.sizeof(L.AzEpisodeStep))
                    o += len(d)
                nu, added = add_from_ranks(replay, allsteps, allgather)
                new_unique += nu
                steps_global += added
            plays += 1
            ss = sp.search.stats()
            sims_done += ss["sims"]
            moves_done += ss["moves"]
            finished += ss["games_finished"]
            games_done += games
            if len(replay) >= min_replay:   # the global length when the buffer is shared
                break
        t1 = time.perf_counter()
        lr = get_cyclical_lr(iteration)
        pl_sum = vl_sum = 0.0
        for b in range(train_steps):
            if shared_replay and shard_batch:     # one global batch, this rank's slice
                planes, pol, val, _ = replay.sample_arrays(batch_size, seed=sample_seed(seed, iteration, b))
                lo, hi = shard_bounds(planes.shape[0], rank, world)
                if hi <= lo:
                    raise ValueError("train: a %d-position batch leaves rank %d no rows" % (planes.shape[0], rank))
            else:
                n = -(-batch_size // world) if shard_batch else batch_size
                planes, pol, val, _ = replay.sample_arrays(n, seed=sample_seed(seed, iteration, b, rank))
                lo, hi = 0, planes.shape[0]
            if log_batch:
                log_batch(iteration, b, planes, pol, val, lo, hi)
            pl, vl = trainer.step(planes[lo:hi], pol[lo:hi], val[lo:hi], lr)
            pl_sum += pl
            vl_sum += vl
        t2 = time.perf_counter()
        st = {"iteration": iteration, "replay": len(replay), "new_unique": new_unique, "lr": lr,
              "policy_loss": pl_sum / max(train_steps, 1), "value_loss": vl_sum / max(train_steps, 1),
              "selfplay_s": t1 - t0, "train_s": t2 - t1, "selfplay_games": games_done, "selfplay_sims": sims_done,
              "games_finished": finished, "episode_steps": steps_done, "moves": moves_done,
              "shared_replay": shared_replay and world > 1, "shard_batch": shard_batch,
              "episode_steps_global": steps_global if shared_replay and world > 1 else steps_done}
        history.append(st)
        if log:
            log(st)
    return trainer, replay, history

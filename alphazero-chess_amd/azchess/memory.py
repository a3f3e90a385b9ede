"""memory.rs mirror: ReplayBuffer (memory.rs:26-117) over libaz's native buffer (az_replay_*).

Same names, argument meaning and error behaviour as the reference: add() returns 1 for a new
unique position and 0 when it folded into an existing entry; sample(batch) returns
min(batch, len) TrainingSamples; save/load use the reference's bincode file layout.
sample() takes a seed (the reference draws from thread_rng); sample_arrays() returns the
batch as the arrays az_trainer_step consumes.
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .chess import Position
from .parameters import REPLAY_BUFFER_SIZE


@dataclass
class TrainingSample:              # memory.rs:11-16
    state: Position
    policy: np.ndarray             # [4096]
    value: float


class ReplayBuffer:
    def __init__(self, capacity=REPLAY_BUFFER_SIZE, _handle=None):
        if _handle is None:
            h = C.c_void_p()
            L.check(L.lib.az_replay_create(int(capacity), C.byref(h)))
            _handle = h
        self._h = _handle
        self.capacity = capacity

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            L.lib.az_replay_destroy(h)
            self._h = None

    def __len__(self):
        return L.check(L.lib.az_replay_len(self._h))

    def len(self):
        return len(self)

    def add(self, step):
        """step: an EpisodeStep (state, improved_policy [4096], final_value) or a raw
        AzEpisodeStep drained from the engine."""
        if isinstance(step, L.AzEpisodeStep):
            return L.check(L.lib.az_replay_add(self._h, C.byref(step)))
        pol = np.ascontiguousarray(step.improved_policy, np.float32)
        assert pol.size == 4096
        return L.check(L.lib.az_replay_add_dense(self._h, C.byref(step.state._p), L.fptr(pol),
                                                 float(step.final_value)))

    def add_many(self, steps):
        """add() every step in order; returns the number of new unique positions.  A ctypes array
        of az_episode_step (unpack_steps, a drain) goes to the engine in one call."""
        if isinstance(steps, C.Array) and issubclass(steps._type_, L.AzEpisodeStep):
            return L.check(L.lib.az_replay_add_many(self._h, steps, len(steps))) if len(steps) else 0
        return sum(self.add(s) for s in steps)

    def sample_arrays(self, batch_size, seed):
        n = min(batch_size, len(self))
        planes = np.empty((n, 19, 64), np.float32)
        pol = np.empty((n, 4096), np.float32)
        val = np.empty(n, np.float32)
        states = (L.AzPos * max(n, 1))()
        got = L.check(L.lib.az_replay_sample(self._h, int(batch_size), C.c_uint64(seed & (2 ** 64 - 1)),
                                             L.fptr(planes), L.fptr(pol), L.fptr(val), states))
        assert got == n
        return planes, pol, val, [Position(L.AzPos.from_buffer_copy(states[i])) for i in range(n)]

    def sample(self, batch_size, seed=0):
        _, pol, val, states = self.sample_arrays(batch_size, seed)
        return [TrainingSample(s, p, float(v)) for s, p, v in zip(states, pol, val)]

    def save(self, path):
        L.check(L.lib.az_replay_save(self._h, str(path).encode()))

    @staticmethod
    def load(path, capacity=REPLAY_BUFFER_SIZE):
        h = C.c_void_p()
        L.check(L.lib.az_replay_load(str(path).encode(), int(capacity), C.byref(h)))
        return ReplayBuffer(capacity, _handle=h)


# ---------------------------------------------------------------- one buffer over the ranks
# The reference keeps ONE replay buffer (memory.rs:41-96) that every self-play task feeds
# (training.rs:81-105).  With one process per GPU every rank keeps a replica: after each self-play
# pass the ranks exchange their drained az_episode_step records and every rank adds the union in
# (rank, drain) order, so the replicas stay byte-identical (same entries, same running means, same
# FIFO order) and a shared sample seed draws the same global batch on every rank.
_STEP_SIZE = C.sizeof(L.AzEpisodeStep)
_HEAD = L.AzEpisodeStep.vis_idx.offset          # game_id .. state: 112 bytes
_NVIS = L.AzEpisodeStep.nvis.offset
_IDX, _CNT = L.AzEpisodeStep.vis_idx.offset, L.AzEpisodeStep.vis_n.offset
_NV = len(L.AzEpisodeStep().vis_idx)


def pack_steps(steps):
    """az_episode_step records -> compact bytes (the header and position of each record, then only
    the nvis live (index, visits) pairs): u64 count | count x 112-byte heads | indices | visits."""
    n = len(steps)
    if n == 0:
        return np.zeros(1, "<u8").tobytes()
    arr = steps if isinstance(steps, C.Array) else (L.AzEpisodeStep * n)(*steps)
    raw = np.frombuffer(arr, np.uint8).reshape(n, _STEP_SIZE)
    nvis = raw[:, _NVIS:_NVIS + 4].copy().view("<i4").ravel()
    if np.any(nvis < 0) or np.any(nvis > _NV):
        raise ValueError("pack_steps: nvis out of range")
    live = np.arange(_NV)[None, :] < nvis[:, None]
    idx = raw[:, _IDX:_IDX + 2 * _NV].copy().view("<u2")[live]
    cnt = raw[:, _CNT:_CNT + 2 * _NV].copy().view("<u2")[live]
    return b"".join([np.array([n], "<u8").tobytes(), raw[:, :_HEAD].tobytes(), idx.tobytes(), cnt.tobytes()])


def unpack_steps(buf):
    """pack_steps' bytes -> a ctypes array of az_episode_step (what az_replay_add takes)."""
    b = np.frombuffer(buf, np.uint8)
    if b.size < 8:
        raise ValueError("unpack_steps: truncated")
    n = int(b[:8].view("<u8")[0])
    heads = b[8:8 + n * _HEAD]
    if heads.size != n * _HEAD:
        raise ValueError("unpack_steps: truncated")
    raw = np.zeros((n, _STEP_SIZE), np.uint8)
    raw[:, :_HEAD] = heads.reshape(n, _HEAD)
    nvis = raw[:, _NVIS:_NVIS + 4].copy().view("<i4").ravel()
    if np.any(nvis < 0) or np.any(nvis > _NV):
        raise ValueError("unpack_steps: nvis out of range")
    tot = int(nvis.sum())
    rest = b[8 + n * _HEAD:]
    if rest.size != 4 * tot:
        raise ValueError("unpack_steps: %d payload bytes for %d visit pairs" % (rest.size, tot))
    live = np.arange(_NV)[None, :] < nvis[:, None]
    idx = np.zeros((n, _NV), "<u2")
    cnt = np.zeros((n, _NV), "<u2")
    idx[live] = rest[:2 * tot].view("<u2")
    cnt[live] = rest[2 * tot:].view("<u2")
    raw[:, _IDX:_IDX + 2 * _NV] = idx.view(np.uint8)
    raw[:, _CNT:_CNT + 2 * _NV] = cnt.view(np.uint8)
    return (L.AzEpisodeStep * n).from_buffer_copy(raw.tobytes()) if n else (L.AzEpisodeStep * 0)()


def add_from_ranks(replay, local_steps, allgather):
    """Every rank's drained steps into this rank's replica, in (rank, drain) order.
    allgather(bytes) -> [bytes of rank 0, ..., rank world-1] (azchess.dist.allgather_bytes, or any
    host transport).  Returns (new unique positions, steps added over all ranks)."""
    parts = allgather(pack_steps(local_steps))
    new = added = 0
    for p in parts:
        steps = unpack_steps(p)
        new += replay.add_many(steps)
        added += len(steps)
    return new, added

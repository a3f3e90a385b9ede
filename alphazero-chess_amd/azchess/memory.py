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

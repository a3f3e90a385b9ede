"""training.rs mirror of the self-play hot path: EpisodeStep, run_episode,
run_all_episodes and process_batch (src/training.rs:15-38, 294-422).

The reference runs one tokio task per game and batches leaf evaluations through an
mpsc channel; here all games of a GPU advance in lockstep inside libaz and every
simulation step evaluates all pending leaves in one batch, with nothing crossing PCIe
until a move's EpisodeSteps are drained.
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .chess import Position, to_tensor
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
        L.check(L.lib.az_selfplay_reset(self.search._h))

    def step(self):
        fin, act = C.c_int(), C.c_int()
        L.check(L.lib.az_selfplay_step(self.search._h, C.byref(fin), C.byref(act)))
        return fin.value, act.value

    def drain(self):
        out = []
        buf = (L.AzEpisodeStep * 4096)()
        while True:
            n = L.check(L.lib.az_selfplay_drain(self.search._h, buf, 4096))
            out += [_convert(buf[i]) for i in range(n)]
            if n < 4096:
                return out


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

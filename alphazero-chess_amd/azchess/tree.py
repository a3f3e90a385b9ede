"""tree.rs mirror: MCTree over the GPU-resident batched search (libaz az_search_*).

`MCTree` is one game's tree with the reference's method names; `BatchedSearch` runs G trees
in lockstep on one GPU (what the engine actually does for self-play).
"""
import ctypes as C

import numpy as np

from . import _lib as L
from .parameters import CACHE_CAPACITY, C_PUCT, DIRICHLET_ALPHA, DIRICHLET_EPSILON, NUM_SIMULATIONS, SEED, TEMPERATURE_ANNEALING


def make_cfg(games, sims=NUM_SIMULATIONS, c_puct=C_PUCT, dir_alpha=DIRICHLET_ALPHA, dir_eps=DIRICHLET_EPSILON,
             temp_moves=TEMPERATURE_ANNEALING, noise=True, seed=SEED, synthetic=False, continuous=False,
             record_evals=False, eval_log_cap=0, cache_capacity=CACHE_CAPACITY):
    return L.AzSearchCfg(games, sims, c_puct, dir_alpha, dir_eps, temp_moves, 1 if noise else 0, seed,
                         L.EVAL_SYNTHETIC if synthetic else L.EVAL_NET, 1 if continuous else 0,
                         1 if record_evals else 0, eval_log_cap, cache_capacity)


class BatchedSearch:
    """G concurrent game trees on one device."""

    def __init__(self, model=None, games=1, device=0, **cfg):
        synthetic = model is None
        self.cfg = make_cfg(games, synthetic=synthetic, **cfg)
        self.games = games
        self.model = model
        h = C.c_void_p()
        L.check(L.lib.az_search_create(model._h if model is not None else None, C.byref(self.cfg), device,
                                       C.byref(h)))
        self._h = h

    def __del__(self):
        try:
            L.lib.az_search_destroy(self._h)
        except Exception:
            pass

    def set_roots(self, histories, apply_noise=False, game_ids=None, noise_plies=None):
        """MCTree::new(eval(root), state, apply_noise) for each game; state = startpos + history."""
        assert len(histories) == self.games
        off = np.zeros(self.games + 1, np.int32)
        for g, h in enumerate(histories):
            off[g + 1] = off[g] + len(h)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(h, np.int32) for h in histories] + [np.zeros(1, np.int32)]))
        gid = np.arange(self.games, dtype=np.int32) if game_ids is None else np.asarray(game_ids, np.int32)
        plies = (off[1:] - off[:-1]).astype(np.int32) if noise_plies is None else np.asarray(noise_plies, np.int32)
        L.check(L.lib.az_search_set_roots(self._h, L.i32ptr(flat), L.i32ptr(off), L.i32ptr(gid), L.i32ptr(plies),
                                          1 if apply_noise else 0))

    def run(self):
        """monte_carlo_tree_search for every game -> (improved [G,4096], visits [G,4096], depth [G])."""
        imp = np.zeros((self.games, 4096), np.float32)
        vis = np.zeros((self.games, 4096), np.uint32)
        dep = np.zeros(self.games, np.int32)
        L.check(L.lib.az_search_run(self._h, L.fptr(imp), L.u32ptr(vis), L.i32ptr(dep)))
        return imp, vis, dep

    def advance(self, actions, apply_noise=True):
        a = np.ascontiguousarray(actions, np.int32)
        res = np.zeros(self.games, np.int32)
        L.check(L.lib.az_search_advance(self._h, L.i32ptr(a), 1 if apply_noise else 0, L.i32ptr(res)))
        return res

    @property
    def persistent(self):
        """True if the untimed simulation steps run through the persistent per-game kernel."""
        return bool(L.lib.az_search_persistent(self._h))

    def stats(self):
        s = L.AzSearchStats()
        L.check(L.lib.az_search_stats_get(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in s._fields_}

    def eval_log(self):
        nr, npri = C.c_int64(), C.c_int64()
        L.check(L.lib.az_search_eval_log(self._h, C.byref(nr), C.byref(npri), None, None, None, None, None))
        keys = np.zeros(max(nr.value, 1), np.uint64)
        vals = np.zeros(max(nr.value, 1), np.float32)
        off = np.zeros(nr.value + 1, np.int32)
        idx = np.zeros(max(npri.value, 1), np.int32)
        pri = np.zeros(max(npri.value, 1), np.float32)
        L.check(L.lib.az_search_eval_log(self._h, C.byref(nr), C.byref(npri), L.u64ptr(keys), L.fptr(vals),
                                         L.i32ptr(off), L.i32ptr(idx), L.fptr(pri)))
        n = nr.value
        return keys[:n], vals[:n], off, idx[:off[n]], pri[:off[n]]

    def timing(self, reset=False, enable=None):
        t = L.AzTiming()
        L.check(L.lib.az_search_timing(self._h, C.byref(t), 1 if reset else 0,
                                       1 if (enable if enable is not None else True) else 0))
        return {k: getattr(t, k) for k, _ in t._fields_}


class MCTree:
    """One game's search tree (tree.rs:25-269), backed by a 1-game BatchedSearch."""

    def __init__(self, search, history):
        self._s = search
        self.history = list(history)

    @classmethod
    def init(cls, model, state, apply_noise, **cfg):
        """MCTree::init (tree.rs:37-64): evaluate the root with `model`."""
        s = BatchedSearch(model, games=1, **cfg)
        hist = list(state.history())
        s.set_roots([hist], apply_noise=apply_noise)
        return cls(s, hist)

    def monte_carlo_tree_search(self):
        """tree.rs:106-115: run the simulations, return the improved policy [4096]."""
        imp, vis, dep = self._s.run()
        self.visits, self.depth = vis[0].astype(np.float32), int(dep[0])
        return imp[0]

    def max_subtree_depth(self):
        return self.depth

    def traverse_new(self, action, apply_noise):
        """tree.rs:239-256 (the action is also played on the tree's GameState)."""
        res = self._s.advance([action], apply_noise=apply_noise)
        self.history.append(int(action))
        return int(res[0])

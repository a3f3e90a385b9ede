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
             record_evals=False, eval_log_cap=0, cache_capacity=CACHE_CAPACITY, callback=False):
    kind = L.EVAL_CALLBACK if callback else (L.EVAL_SYNTHETIC if synthetic else L.EVAL_NET)
    return L.AzSearchCfg(games, sims, c_puct, dir_alpha, dir_eps, temp_moves, 1 if noise else 0, seed,
                         kind, 1 if continuous else 0, 1 if record_evals else 0, eval_log_cap, cache_capacity)


def _eval_trampoline(evaluator):
    """az_eval_fn around a Python process_batch-style callable (training.rs:380-422):
    evaluator(positions) -> (policy [n, 4096], value [n]); its rows are copied into the engine's
    staging buffers."""
    from .chess import Position

    def fn(_ctx, pos, n, pol, val):
        try:
            states = [Position(L.AzPos.from_buffer_copy(pos[i])) for i in range(n)]
            p, v = evaluator(states)
            np.ctypeslib.as_array(pol, shape=(n * 4096,))[:] = np.asarray(p, np.float32).reshape(n * 4096)
            np.ctypeslib.as_array(val, shape=(n,))[:] = np.asarray(v, np.float32).reshape(n)
            return 0
        except BaseException as e:              # nothing may unwind through the C frames, not even
            import traceback                    # KeyboardInterrupt / SystemExit (ctypes would swallow
            traceback.print_exc()               # them and report success over stale staging rows)
            if not isinstance(e, Exception):
                pending[0] = e
            return 1
    pending = [None]
    return L.EVAL_FN(fn), pending


class BatchedSearch:
    """G concurrent game trees on one device."""

    def __init__(self, model=None, games=1, device=0, evaluator=None, **cfg):
        """model: an AlphaZero (AZ_EVAL_NET); evaluator: a caller-owned process_batch-style callable
        (AZ_EVAL_CALLBACK); neither: the synthetic evaluator the oracle shares."""
        synthetic = model is None and evaluator is None
        self.cfg = make_cfg(games, synthetic=synthetic, callback=evaluator is not None, **cfg)
        self.games = games
        self.model = model
        h = C.c_void_p()
        L.check(L.lib.az_search_create(model._h if model is not None else None, C.byref(self.cfg), device,
                                       C.byref(h)))
        self._h = h
        self._eval_fn, self._pending = None, [None]
        if evaluator is not None:
            self._eval_fn, self._pending = _eval_trampoline(evaluator)     # kept alive as long as the engine
            L.check(L.lib.az_search_set_evaluator(self._h, C.cast(self._eval_fn, C.c_void_p), None))

    def __del__(self):
        try:
            L.lib.az_search_destroy(self._h)
        except Exception:
            pass

    def check(self, rc):
        """L.check for calls that may run the caller's evaluator: a KeyboardInterrupt / SystemExit
        raised inside it is re-raised here, after the C call has returned its error."""
        e, self._pending[0] = self._pending[0], None
        if e is not None:
            raise e
        return L.check(rc)

    def set_roots(self, histories, apply_noise=False, game_ids=None, noise_plies=None, start=None):
        """MCTree::new(eval(root), state, apply_noise) for each game; state = start + history
        (start: a list of G Positions, e.g. from FENs; None = the startpos)."""
        assert len(histories) == self.games
        off = np.zeros(self.games + 1, np.int32)
        for g, h in enumerate(histories):
            off[g + 1] = off[g] + len(h)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(h, np.int32) for h in histories] + [np.zeros(1, np.int32)]))
        gid = np.arange(self.games, dtype=np.int32) if game_ids is None else np.asarray(game_ids, np.int32)
        plies = (off[1:] - off[:-1]).astype(np.int32) if noise_plies is None else np.asarray(noise_plies, np.int32)
        st = None
        if start is not None:
            assert len(start) == self.games
            st = (L.AzPos * self.games)()
            for g, p in enumerate(start):
                st[g] = p._p
        self.check(L.lib.az_search_set_roots_from(self._h, st, L.i32ptr(flat), L.i32ptr(off), L.i32ptr(gid),
                                               L.i32ptr(plies), 1 if apply_noise else 0))

    def run(self):
        """monte_carlo_tree_search for every game -> (improved [G,4096], visits [G,4096], depth [G])."""
        imp = np.zeros((self.games, 4096), np.float32)
        vis = np.zeros((self.games, 4096), np.uint32)
        dep = np.zeros(self.games, np.int32)
        self.check(L.lib.az_search_run(self._h, L.fptr(imp), L.u32ptr(vis), L.i32ptr(dep)))
        return imp, vis, dep

    def read_roots(self):
        """(improved [G,4096], visits [G,4096], depth [G]) of the current roots, no simulations run
        (the reference's public MCTree fields, tree.rs:25-34)."""
        imp = np.zeros((self.games, 4096), np.float32)
        vis = np.zeros((self.games, 4096), np.uint32)
        dep = np.zeros(self.games, np.int32)
        L.check(L.lib.az_search_read_roots(self._h, L.fptr(imp), L.u32ptr(vis), L.i32ptr(dep)))
        return imp, vis, dep

    def advance(self, actions, apply_noise=True):
        a = np.ascontiguousarray(actions, np.int32)
        res = np.zeros(self.games, np.int32)
        self.check(L.lib.az_search_advance(self._h, L.i32ptr(a), 1 if apply_noise else 0, L.i32ptr(res)))
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

"""validation.rs / ratings.rs mirror: the evaluation arena and Elo ratings.

`evaluate(player_1, player_2)` is validation.rs:155-282 + play_evaluation_game (:284-402): G games
in lockstep, player_1 White in the even games and Black in the odd ones; an MCTS player searches
a fresh tree from the current position every move (MCTree::async_init(.., false): no noise, no
subtree reuse) -- all of that player's games to move go through ONE BatchedSearch on the GPU;
a base-model player takes the network's policy masked to the legal moves; a random player picks
uniformly from the legal-move list (under-promotions included as separate entries).
Move choice: argmax (Rust max_by: the LAST maximal index) once fullmoves > num_stochastic_moves,
else rand 0.8 WeightedIndex over the policy (float32 cumulative sums).  thread_rng is replaced by
a seeded stream per (seed, game, ply) so a match is reproducible.
`compute_elo_rankings` / `compute_elos` are ratings.rs:5-28 and :113-143 (float32, 1000
iterations of rate 8, player 0 pinned at the base Elo).
The minimax and human players (chess.rs:248-420, validation.rs:91-117) are out of scope.
"""
from dataclasses import dataclass

import numpy as np

from .chess import GameState, play_move, to_tensor
from .parameters import EVALUATION_GAMES, NUM_SIMULATIONS, TEMPERATURE_ANNEALING
from .tree import BatchedSearch


@dataclass
class EvaluationResult:             # validation.rs:12-19
    num_inferences: float
    avg_batch_size: float
    winrate: float
    p1_winrate: float
    p2_winrate: float
    drawrate: float


class Player:                       # validation.rs:21-27 (MctsModel, BaseModel, Random)
    def __init__(self, kind, model=None):
        assert kind in ("mcts", "base", "random")
        self.kind, self.model = kind, model

    @staticmethod
    def mcts(model):
        """Player::MctsModel; model=None searches with libaz's synthetic evaluator (tests)."""
        return Player("mcts", model)

    @staticmethod
    def base(model):
        return Player("base", model)

    @staticmethod
    def random():
        return Player("random")


def argmax_last(v):
    """Iterator::enumerate().max_by(partial_cmp): the last index among equal maxima."""
    v = np.asarray(v, np.float32)
    return int(len(v) - 1 - np.argmax(v[::-1]))


def weighted_index(w, u):
    """rand 0.8 WeightedIndex::new(w).sample(): cumulative float32 sums; x = u * total;
    the first index whose cumulative weight exceeds x."""
    w = np.asarray(w, np.float32)
    cum = np.cumsum(w, dtype=np.float32)           # sequential float32 accumulation
    total = cum[-1]
    x = np.float32(np.float32(u) * total)
    if not x < total:
        x = np.nextafter(total, np.float32(0))
    return int(np.searchsorted(cum[:-1], x, side="right"))


def choice_uniform(seed, game, ply):
    """u in [0, 1) (float32) for the move choice of (game, ply): the seeded thread_rng stand-in."""
    return np.float32(np.random.default_rng([seed, game, ply]).random(dtype=np.float32))


def choose(policy, fullmoves, num_stochastic_moves, u):
    if fullmoves > num_stochastic_moves:          # validation.rs:297 (strictly greater)
        return argmax_last(policy)
    return weighted_index(policy, u)


def evaluate(player_1, player_2, games=EVALUATION_GAMES, sims=NUM_SIMULATIONS,
             num_stochastic_moves=TEMPERATURE_ANNEALING, seed=0, device=0, max_plies=1000, record=False):
    """validation.rs:155-282.  Returns EvaluationResult (and the games' move lists and results
    when record=True)."""
    G = games
    states = [GameState() for _ in range(G)]
    hist = [[] for _ in range(G)]
    result = [None] * G                           # White's result: 1, 0, -1
    # a player moves in at most half of the games at once, or in all of them when it plays both
    # colours (player_1 is player_2)
    slots = G if player_1 is player_2 else (G + 1) // 2
    searches = {}
    for p in (player_1, player_2):
        if p.kind == "mcts" and id(p) not in searches:
            searches[id(p)] = BatchedSearch(p.model, games=slots, device=device, sims=sims, noise=False,
                                            cache_capacity=0)
    num_inferences, rows = 0, 0
    for ply in range(max_plies):
        live = [g for g in range(G) if result[g] is None]
        if not live:
            break
        white_to_move = ply % 2 == 0
        by_player = {}
        for g in live:
            white = player_1 if g % 2 == 0 else player_2
            black = player_2 if g % 2 == 0 else player_1
            p = white if white_to_move else black
            by_player.setdefault(id(p), (p, []))[1].append(g)
        actions = {}
        for p, gs in by_player.values():
            if p.kind == "random":
                rng = np.random.default_rng([seed, ply, 7])
                for g in gs:
                    legal = states[g].position.legal_indices()   # with under-promotion duplicates
                    actions[g] = int(legal[rng.integers(len(legal))])
                continue
            if p.kind == "mcts":
                s = searches[id(p)]
                roots = [hist[g] for g in gs] + [hist[gs[0]]] * (slots - len(gs))   # pad with a live root
                e0 = s.stats()["evals"]
                s.set_roots(roots, apply_noise=False)
                imp, _, _ = s.run()
                pols = imp[:len(gs)]
                num_inferences += sims + 1               # root batch + one batch per simulation step
                rows += s.stats()["evals"] - e0
            else:
                x = np.concatenate([to_tensor(states[g].position) for g in gs], 0)
                pol, _ = p.model.forward(x)
                num_inferences += 1
                rows += len(gs)
                pols = np.zeros_like(pol)
                for k, g in enumerate(gs):
                    legal = np.unique(states[g].position.legal_indices())
                    pols[k, legal] = pol[k, legal]            # validation.rs:327-331
            for k, g in enumerate(gs):
                actions[g] = choose(pols[k], states[g].position.fullmoves, num_stochastic_moves,
                                    choice_uniform(seed, g, ply))
        for g in live:
            r = int(play_move(states[g], actions[g]))
            hist[g].append(actions[g])
            if r == 1:
                result[g] = 0
            elif r == 2:
                result[g] = 1
            elif r == 3:
                result[g] = -1
            elif r != 0:
                raise RuntimeError("player played an illegal move")
    p1_score = [(r if g % 2 == 0 else -r) for g, r in enumerate(result) if r is not None]
    p1_wins = sum(1 for r in p1_score if r > 0)
    draws = sum(1 for r in p1_score if r == 0)
    res = EvaluationResult(float(num_inferences), rows / max(num_inferences, 1),
                           (p1_wins + draws / 2.0) / G, p1_wins / G, (G - p1_wins - draws) / G, draws / G)
    if record:
        return res, hist, result
    return res


def compute_elos(winrate_matrix, base_elo):
    """ratings.rs:113-143 in float32."""
    wm = np.asarray(winrate_matrix, np.float32)
    n = len(wm)
    f = np.float32
    elos = np.full(n, f(base_elo), np.float32)
    for _ in range(1000):
        prev = elos.copy()
        for i in range(1, n):
            actual, expected = f(0.0), f(0.0)
            for j in range(n):
                if i == j:
                    continue
                actual = f(actual + wm[i][j])
                diff = f(prev[j] - prev[i])
                expected = f(expected + f(1.0) / (f(1.0) + np.power(f(10.0), f(diff / f(400.0)))))
            elos[i] = f(elos[i] + f(8.0) * f(actual - expected))
    return elos


def compute_elo_rankings(players, base_elo=150.0, **kw):
    """ratings.rs:5-28: round robin, winrate matrix, Elo.  Returns (avg_batch_size, elos, matrix)."""
    n = len(players)
    wm = [[0.5] * n for _ in range(n)]
    ninf, avg = 0.0, 0.0
    for i in range(n):
        for j in range(i):
            r = evaluate(players[i], players[j], **kw)
            avg = r.avg_batch_size * r.num_inferences + avg * ninf
            ninf += r.num_inferences
            avg /= max(ninf, 1.0)
            wm[j][i] = 1.0 - r.winrate
            wm[i][j] = r.winrate
    return avg, compute_elos(wm, base_elo), wm

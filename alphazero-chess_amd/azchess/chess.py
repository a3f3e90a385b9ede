"""chess.rs mirror over libaz: GameState, GameResult, play_move, move_to_index,
index_to_move, to_tensor (AlexandreGac/alphazero-chess src/chess.rs).

Moves are represented by their policy index (0..4095) -- the reference's index_to_move
(chess.rs:118-171) is exactly the bridge the search uses, so `index_to_move(i, pos)` returns
`i` itself when legal (None otherwise) and `play_move` takes that index.
"""
import ctypes as C
import enum

import numpy as np

from . import _lib as L


class GameResult(enum.IntEnum):      # chess.rs:29-34
    Ongoing = L.ONGOING
    Draw = L.DRAW
    WhiteWins = L.WHITE_WINS
    BlackWins = L.BLACK_WINS


class IllegalMove(ValueError):
    pass


class Position:
    """shakmaty::Chess replacement: an 80-byte az_pos."""

    __slots__ = ("_p",)

    def __init__(self, raw=None):
        self._p = raw if raw is not None else L.AzPos()

    @staticmethod
    def startpos():
        p = Position()
        L.check(L.lib.az_pos_startpos(C.byref(p._p)))
        return p

    @staticmethod
    def from_fen(fen):
        p = Position()
        L.check(L.lib.az_pos_from_fen(fen.encode(), C.byref(p._p)))
        return p

    def fen(self):
        buf = C.create_string_buffer(128)
        L.check(L.lib.az_pos_to_fen(C.byref(self._p), buf, 128))
        return buf.value.decode()

    def fen_key(self):
        return int(L.lib.az_pos_fen_key(C.byref(self._p)))

    @property
    def turn(self):                  # 0 White, 1 Black
        return int(self._p.turn)

    @property
    def halfmoves(self):
        return int(self._p.halfmoves)

    @property
    def fullmoves(self):
        return int(self._p.fullmoves)

    def bitboards(self):
        return np.array(list(self._p.bb), dtype=np.uint64)

    def legal_indices(self):
        out = np.zeros(L.MAX_MOVES, np.int32)
        n = L.check(L.lib.az_pos_legal_indices(C.byref(self._p), L.i32ptr(out), L.MAX_MOVES))
        return out[:n].copy()

    def play(self, index):
        c = Position()
        if not L.lib.az_pos_play_index(C.byref(self._p), int(index), C.byref(c._p)):
            raise IllegalMove(index)
        return c

    def outcome(self):
        return GameResult(L.check(L.lib.az_pos_outcome(C.byref(self._p))))

    def raw(self):
        return bytes(self._p)

    def __eq__(self, other):
        return isinstance(other, Position) and bytes(self._p) == bytes(other._p)

    def __repr__(self):
        return "Position(%r)" % self.fen()


class GameState:
    """chess.rs:13-27 -- position + repetition multiset (kept as the full history)."""

    def __init__(self, _handle=None):
        h = C.c_void_p()
        if _handle is None:
            L.check(L.lib.az_game_create(C.byref(h)))
        else:
            h = _handle
        self._h = h

    def __del__(self):
        try:
            L.lib.az_game_destroy(self._h)
        except Exception:
            pass

    def clone(self):
        h = C.c_void_p()
        L.check(L.lib.az_game_clone(self._h, C.byref(h)))
        return GameState(h)

    @property
    def position(self):
        p = Position()
        L.check(L.lib.az_game_position(self._h, C.byref(p._p)))
        return p

    def history(self):
        n = L.check(L.lib.az_game_history(self._h, None, 0))
        out = np.zeros(max(n, 1), np.int32)
        L.lib.az_game_history(self._h, L.i32ptr(out), n)
        return out[:n].copy()


def play_move(state, action):
    """chess.rs:36-63: returns GameResult or raises IllegalMove (Err("Illegal move"))."""
    r = L.lib.az_game_play(state._h, int(action))
    if r == L.ILLEGAL:
        raise IllegalMove(action)
    return GameResult(r)


def move_to_index(from_sq, to_sq, turn):
    """chess.rs:73-116 (castling: to_sq = rook square, shakmaty Move::to())."""
    return int(L.lib.az_move_to_index(int(from_sq), int(to_sq), int(turn)))


def index_to_move(index, position):
    """chess.rs:118-171: Some(index) if it names a legal move of `position`, else None."""
    c = L.AzPos()
    return int(index) if L.lib.az_pos_play_index(C.byref(position._p), int(index), C.byref(c)) else None


def to_tensor(position):
    """chess.rs:191-245: [1,19,8,8] float32 in the side-to-move frame."""
    t = np.zeros((1, 19, 8, 8), np.float32)
    L.check(L.lib.az_pos_encode(C.byref(position._p), L.fptr(t)))
    return t


def positions_to_array(positions):
    """a numpy az_pos array (L.POS_DTYPE) from Positions"""
    out = np.zeros(len(positions), L.POS_DTYPE)
    buf = out.view(np.uint8).reshape(len(positions), 80)
    for i, p in enumerate(positions):
        buf[i] = np.frombuffer(bytes(p._p), np.uint8)
    return out


def array_position(arr, i):
    """Position i of a numpy az_pos array"""
    return Position(L.AzPos.from_buffer_copy(arr[i:i + 1].tobytes()))


def rules_probe(parents, actions, device=0):
    """az_rules_probe (test hook): the device rules path on items (parent, action) -- action < 0
    probes the parent itself.  parents: a numpy az_pos array (L.POS_DTYPE) or a list of Positions.
    Returns a dict: child (az_pos array), moves [n,256] / nmoves [n] (leaf generator, duplicates
    included), root_moves / root_n (the roots' generator), outcome, in_check, fen_key, planes
    [n,19,8,8]."""
    if not isinstance(parents, np.ndarray):
        parents = positions_to_array(parents)
    par = np.ascontiguousarray(parents, L.POS_DTYPE)
    n = len(par)
    act = np.ascontiguousarray(actions, np.int32)
    assert len(act) == n
    child = np.zeros(n, L.POS_DTYPE)
    mv = np.zeros((n, L.MAX_MOVES), np.int32)
    nm = np.zeros(n, np.int32)
    rmv = np.zeros((n, L.MAX_MOVES), np.int32)
    rn = np.zeros(n, np.int32)
    oc = np.zeros(n, np.int32)
    chk = np.zeros(n, np.int32)
    fk = np.zeros(n, np.uint64)
    planes = np.zeros((n, 19, 8, 8), np.float32)
    pp = lambda a: a.ctypes.data_as(C.POINTER(L.AzPos))
    L.check(L.lib.az_rules_probe(device, pp(par), L.i32ptr(act), n, pp(child), L.i32ptr(mv), L.i32ptr(nm),
                                 L.i32ptr(rmv), L.i32ptr(rn), L.i32ptr(oc), L.i32ptr(chk), L.u64ptr(fk),
                                 L.fptr(planes)))
    return dict(child=child, moves=mv, nmoves=nm, root_moves=rmv, root_n=rn, outcome=oc, in_check=chk,
                fen_key=fk, planes=planes)

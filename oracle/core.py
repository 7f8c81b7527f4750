"""TEST INFRASTRUCTURE ONLY — ctypes wrapper over oracle/liboracle.so.

Each wrapper names the reference code it restates (see uttt_oracle.c for the
file:line of every function).
"""
import ctypes
import os

import numpy as np

from . import ORACLE_DIR

_LIB = None

I32P = ctypes.POINTER(ctypes.c_int32)
F32P = ctypes.POINTER(ctypes.c_float)
F64P = ctypes.POINTER(ctypes.c_double)


class OrState(ctypes.Structure):
    """cpp/uttt_game.h:11-59 State (int arrays, side-to-move relative)."""

    _fields_ = [
        ("pieces", (ctypes.c_int32 * 9) * 9),
        ("enemy", (ctypes.c_int32 * 9) * 9),
        ("main_p", ctypes.c_int32 * 9),
        ("main_e", ctypes.c_int32 * 9),
        ("active", ctypes.c_int32),
    ]

    @classmethod
    def initial(cls):
        s = cls()
        lib().or_state_initial(ctypes.byref(s))
        return s

    @classmethod
    def from_arrays(cls, pieces, enemy, main_p, main_e, active):
        s = cls()
        p = np.asarray(pieces, dtype=np.int32).reshape(9, 9)
        e = np.asarray(enemy, dtype=np.int32).reshape(9, 9)
        for b in range(9):
            for c in range(9):
                s.pieces[b][c] = int(p[b, c])
                s.enemy[b][c] = int(e[b, c])
        for i in range(9):
            s.main_p[i] = int(main_p[i])
            s.main_e[i] = int(main_e[i])
        s.active = int(active)
        return s

    def arrays(self):
        p = np.array([[self.pieces[b][c] for c in range(9)] for b in range(9)], dtype=np.int32)
        e = np.array([[self.enemy[b][c] for c in range(9)] for b in range(9)], dtype=np.int32)
        return (p, e, np.array(list(self.main_p), np.int32), np.array(list(self.main_e), np.int32),
                int(self.active))

    def legal_actions(self):
        out = (ctypes.c_int32 * 81)()
        n = lib().or_legal_actions(ctypes.byref(self), out)
        return [out[i] for i in range(n)]

    def next(self, action):
        o = OrState()
        lib().or_next(ctypes.byref(self), int(action), ctypes.byref(o))
        return o

    def is_lose(self):
        return bool(lib().or_is_lose(ctypes.byref(self)))

    def is_draw(self):
        return bool(lib().or_is_draw(ctypes.byref(self)))

    def is_done(self):
        return bool(lib().or_is_done(ctypes.byref(self)))

    def is_first_player(self):
        return bool(lib().or_is_first_player(ctypes.byref(self)))

    def tensor_hwc(self):
        t = np.zeros(243, np.float32)
        lib().or_tensor_hwc(ctypes.byref(self), t.ctypes.data_as(F32P))
        return t

    def tensor_nchw(self):
        t = np.zeros(243, np.float32)
        lib().or_tensor_nchw(ctypes.byref(self), t.ctypes.data_as(F32P))
        return t


class SearchStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("flushes", "evals", "terminal", "max_depth", "nodes", "max_children")]


EVAL_FN = ctypes.CFUNCTYPE(None, F32P, F32P, F32P, ctypes.c_void_p)


class MT(ctypes.Structure):
    """numpy legacy RandomState MT19937 state."""

    _fields_ = [("key", ctypes.c_uint32 * 624), ("pos", ctypes.c_int32)]

    def __init__(self, seed=0):
        super().__init__()
        lib().or_mt_seed(ctypes.byref(self), ctypes.c_uint32(seed))

    def next32(self):
        return lib().or_mt_next32(ctypes.byref(self))

    def double(self):
        return lib().or_mt_double(ctypes.byref(self))


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            from . import build
            build()
        L = ctypes.CDLL(path)
        sp = ctypes.POINTER(OrState)
        L.or_state_initial.argtypes = [sp]
        L.or_legal_actions.argtypes = [sp, I32P]
        L.or_next.argtypes = [sp, ctypes.c_int, sp]
        for f in ("or_is_lose", "or_is_draw", "or_is_done", "or_is_first_player"):
            getattr(L, f).argtypes = [sp]
        L.or_tensor_hwc.argtypes = [sp, F32P]
        L.or_tensor_nchw.argtypes = [sp, F32P]
        L.or_hash_eval.argtypes = [F32P, F32P, F32P]
        L.or_pv_mcts_scores.argtypes = [sp, ctypes.c_float, ctypes.c_int, ctypes.c_int, EVAL_FN,
                                        ctypes.c_void_p, F32P, I32P, ctypes.POINTER(SearchStats)]
        L.or_pv_mcts_scores_hash.argtypes = [sp, ctypes.c_float, ctypes.c_int, ctypes.c_int, F32P, I32P,
                                             ctypes.POINTER(SearchStats)]
        L.or_boltzman.argtypes = [F32P, ctypes.c_int, ctypes.c_float, F32P]
        L.or_pv_mcts_scores_py.argtypes = [sp, ctypes.c_double, ctypes.c_int, ctypes.c_int, EVAL_FN,
                                           ctypes.c_void_p, F64P, I32P, ctypes.POINTER(SearchStats)]
        L.or_pv_mcts_scores_py_hash.argtypes = [sp, ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                                F64P, I32P, ctypes.POINTER(SearchStats)]
        L.or_evaluate_play_hash.argtypes = [ctypes.c_uint32, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_uint64, ctypes.c_uint64, I32P, I32P]
        L.or_self_play_game_py_hash.argtypes = [ctypes.c_uint32, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_uint64, F32P, F64P, ctypes.POINTER(ctypes.c_int8),
                                                ctypes.c_int]
        L.or_np_pairwise_sum_f32.argtypes = [F32P, ctypes.c_int64]
        L.or_np_pairwise_sum_f32.restype = ctypes.c_float
        L.or_mt_seed.argtypes = [ctypes.POINTER(MT), ctypes.c_uint32]
        L.or_mt_next32.argtypes = [ctypes.POINTER(MT)]
        L.or_mt_next32.restype = ctypes.c_uint32
        L.or_mt_double.argtypes = [ctypes.POINTER(MT)]
        L.or_mt_double.restype = ctypes.c_double
        L.or_np_pairwise_sum.argtypes = [F64P, ctypes.c_int64]
        L.or_np_pairwise_sum.restype = ctypes.c_double
        L.or_np_choice.argtypes = [ctypes.POINTER(MT), F64P, ctypes.c_int]
        L.or_policy_and_sample.argtypes = [ctypes.POINTER(MT), F32P, ctypes.c_int, F64P]
        L.or_self_play_game_hash.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, F32P, F64P, I32P, I32P]
        _LIB = L
    return _LIB


def hash_eval(x_nchw):
    """Deterministic hash evaluator on one NCHW (3,9,9) input -> (policy[81] f32, value f32)."""
    x = np.ascontiguousarray(x_nchw, dtype=np.float32).reshape(243)
    pol = np.zeros(81, np.float32)
    v = np.zeros(1, np.float32)
    lib().or_hash_eval(x.ctypes.data_as(F32P), pol.ctypes.data_as(F32P), v.ctypes.data_as(F32P))
    return pol, v[0]


def pv_mcts_scores_hash(state, temperature, evaluate_count=50, batch_size=8):
    """uttt_mcts.cpp:84-196 with the hash evaluator -> (scores f32, visits i32, stats)."""
    sc = np.zeros(81, np.float32)
    vi = np.zeros(81, np.int32)
    st = SearchStats()
    n = lib().or_pv_mcts_scores_hash(ctypes.byref(state), float(temperature), int(evaluate_count),
                                     int(batch_size), sc.ctypes.data_as(F32P), vi.ctypes.data_as(I32P),
                                     ctypes.byref(st))
    return sc[:n].copy(), vi[:n].copy(), st


def pv_mcts_scores(state, temperature, evaluate_count, batch_size, evaluator):
    """Search with a Python evaluator: evaluator(x_nchw (243,) f32) -> (policy[81], value)."""

    def cb(xp, pp, vp, _ctx):
        x = np.ctypeslib.as_array(xp, shape=(243,)).copy()
        pol, val = evaluator(x)
        pol = np.asarray(pol, dtype=np.float32).reshape(-1)
        for a in range(81):
            pp[a] = float(pol[a]) if a < pol.size else 0.0
        vp[0] = float(np.float32(val))

    fn = EVAL_FN(cb)
    sc = np.zeros(81, np.float32)
    vi = np.zeros(81, np.int32)
    st = SearchStats()
    n = lib().or_pv_mcts_scores(ctypes.byref(state), float(temperature), int(evaluate_count), int(batch_size),
                                fn, None, sc.ctypes.data_as(F32P), vi.ctypes.data_as(I32P), ctypes.byref(st))
    return sc[:n].copy(), vi[:n].copy(), st


def pv_mcts_scores_py_hash(state, temperature, evaluate_count=50, batch_size=8, salt=0):
    """pv_mcts.py (Python semantics) with the (salted) hash evaluator -> (scores f64, visits i32, stats).
    scores is None where the reference raises ZeroDivisionError (no root child visited)."""
    sc = np.zeros(81, np.float64)
    vi = np.zeros(81, np.int32)
    st = SearchStats()
    n = lib().or_pv_mcts_scores_py_hash(ctypes.byref(state), float(temperature), int(evaluate_count),
                                        int(batch_size), ctypes.c_uint64(salt), sc.ctypes.data_as(F64P),
                                        vi.ctypes.data_as(I32P), ctypes.byref(st))
    vis = vi[:n].copy()
    if temperature != 0 and vis.sum() == 0:
        return None, vis, st
    return sc[:n].copy(), vis, st


def pv_mcts_scores_py_callback(state, temperature, evaluate_count, batch_size, evaluator):
    """pv_mcts.py semantics with a Python evaluator(x_nchw (243,) f32) -> (policy[81], value)."""

    def cb(xp, pp, vp, _ctx):
        x = np.ctypeslib.as_array(xp, shape=(243,)).copy()
        pol, val = evaluator(x)
        pol = np.asarray(pol, dtype=np.float32).reshape(-1)
        for a in range(81):
            pp[a] = float(pol[a]) if a < pol.size else 0.0
        vp[0] = float(np.float32(val))

    fn = EVAL_FN(cb)
    sc = np.zeros(81, np.float64)
    vi = np.zeros(81, np.int32)
    st = SearchStats()
    n = lib().or_pv_mcts_scores_py(ctypes.byref(state), float(temperature), int(evaluate_count), int(batch_size),
                                   fn, None, sc.ctypes.data_as(F64P), vi.ctypes.data_as(I32P), ctypes.byref(st))
    return sc[:n].copy(), vi[:n].copy(), st


def evaluate_play_hash(seed, salt_first, salt_second, temperature=1.0, evaluate_count=50, batch_size=8):
    """evaluate_network.play after np.random.seed(seed), first player = hash(salt_first).
    Returns (first player's point 0 / 0.5 / 1, actions)."""
    acts = np.zeros(81, np.int32)
    na = ctypes.c_int32()
    r = lib().or_evaluate_play_hash(ctypes.c_uint32(seed), float(temperature), int(evaluate_count), int(batch_size),
                                    ctypes.c_uint64(salt_first), ctypes.c_uint64(salt_second),
                                    acts.ctypes.data_as(I32P), ctypes.byref(na))
    if r < 0:
        raise RuntimeError("or_evaluate_play_hash: scores / legal length mismatch")
    return r / 2.0, acts[:na.value].copy()


def self_play_game_py_hash(seed, temperature=1.0, evaluate_count=50, batch_size=8, salt=0, max_plies=81):
    """self_play.py play() after np.random.seed(seed), hash evaluator -> dict of per-ply arrays."""
    t = np.zeros((max_plies, 243), np.float32)
    p = np.zeros((max_plies, 81), np.float64)
    v = np.zeros(max_plies, np.int8)
    n = lib().or_self_play_game_py_hash(ctypes.c_uint32(seed), float(temperature), int(evaluate_count),
                                        int(batch_size), ctypes.c_uint64(salt), t.ctypes.data_as(F32P),
                                        p.ctypes.data_as(F64P), v.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
                                        max_plies)
    if n < 0:
        raise RuntimeError("or_self_play_game_py_hash failed")
    return {"tensors": t[:n], "policies": p[:n], "values": v[:n]}


def np_pairwise_sum_f32(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return np.float32(lib().or_np_pairwise_sum_f32(a.ctypes.data_as(F32P), a.size))


def boltzman(xs, temperature):
    xs = np.ascontiguousarray(xs, dtype=np.float32)
    out = np.zeros_like(xs)
    lib().or_boltzman(xs.ctypes.data_as(F32P), xs.size, float(temperature), out.ctypes.data_as(F32P))
    return out


def np_pairwise_sum(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().or_np_pairwise_sum(a.ctypes.data_as(F64P), a.size)


def policy_and_sample(mt, scores):
    """self_play_cpp.py:74-86 -> (policy over legal f64, sampled index into legal)."""
    scores = np.ascontiguousarray(scores, dtype=np.float32)
    pol = np.zeros(scores.size, np.float64)
    idx = lib().or_policy_and_sample(ctypes.byref(mt), scores.ctypes.data_as(F32P), scores.size,
                                     pol.ctypes.data_as(F64P))
    return pol, idx


def self_play_game_hash(seed, temperature=1.0, evaluate_count=50, batch_size=8, max_plies=81):
    """self_play_cpp.play with RandomState(seed) and the hash evaluator."""
    t = np.zeros((max_plies, 243), np.float32)
    p = np.zeros((max_plies, 81), np.float64)
    a = np.zeros(max_plies, np.int32)
    v = np.zeros(max_plies, np.int32)
    n = lib().or_self_play_game_hash(ctypes.c_uint32(seed), float(temperature), int(evaluate_count),
                                     int(batch_size), max_plies, t.ctypes.data_as(F32P), p.ctypes.data_as(F64P),
                                     a.ctypes.data_as(I32P), v.ctypes.data_as(I32P))
    if n < 0:
        raise RuntimeError(f"oracle self-play failed ({n})")
    return {"tensors": t[:n], "policies": p[:n], "actions": a[:n], "values": v[:n]}

"""TEST INFRASTRUCTURE ONLY — ctypes wrapper over oracle/_ref/libuttt_ref.so.

That library is the reference's own cpp/uttt_game.cpp + cpp/uttt_mcts.cpp,
compiled from the reference checkout by oracle/Makefile, plus oracle/ref_driver.cpp.
It exists only where it was built (the build container, and the GPU box via the
snapshot); callers must handle :func:`available` being False.
"""
import ctypes
import os

import numpy as np

from . import ORACLE_DIR

REF_DIR = os.path.join(ORACLE_DIR, "_ref")
_LIB = None
I32P = ctypes.POINTER(ctypes.c_int32)
F32P = ctypes.POINTER(ctypes.c_float)
I64P = ctypes.POINTER(ctypes.c_int64)


def available():
    return os.path.exists(os.path.join(REF_DIR, "libuttt_ref.so"))


def lib():
    global _LIB
    if _LIB is None:
        L = ctypes.CDLL(os.path.join(REF_DIR, "libuttt_ref.so"))
        st = [I32P, I32P, I32P, I32P, ctypes.c_int32]
        L.ref_legal_actions.argtypes = st + [I32P]
        L.ref_flags.argtypes = st
        L.ref_next.argtypes = st + [ctypes.c_int32, I32P, I32P, I32P, I32P, I32P]
        L.ref_tensor.argtypes = st + [F32P]
        L.ref_to_string.argtypes = st + [ctypes.c_char_p, ctypes.c_int]
        L.ref_search_hash.argtypes = st + [ctypes.c_float, ctypes.c_int, ctypes.c_int, F32P, I64P]
        L.ref_boltzman.argtypes = [F32P, ctypes.c_int, ctypes.c_float, F32P]
        L.ref_bench_tree.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, I64P]
        L.ref_bench_tree.restype = ctypes.c_double
        _LIB = L
    return _LIB


def _args(state):
    p, e, m, me, a = state
    p = np.ascontiguousarray(p, np.int32).reshape(81)
    e = np.ascontiguousarray(e, np.int32).reshape(81)
    m = np.ascontiguousarray(m, np.int32).reshape(9)
    me = np.ascontiguousarray(me, np.int32).reshape(9)
    keep = (p, e, m, me)
    return keep, [p.ctypes.data_as(I32P), e.ctypes.data_as(I32P), m.ctypes.data_as(I32P),
                  me.ctypes.data_as(I32P), int(a)]


def legal_actions(state):
    keep, a = _args(state)
    out = np.zeros(81, np.int32)
    n = lib().ref_legal_actions(*a, out.ctypes.data_as(I32P))
    return out[:n].tolist()


def flags(state):
    """bit0 is_lose, bit1 is_draw, bit2 is_done, bit3 is_first_player."""
    keep, a = _args(state)
    return lib().ref_flags(*a)


def next_state(state, action):
    keep, a = _args(state)
    op = np.zeros(81, np.int32)
    oe = np.zeros(81, np.int32)
    om = np.zeros(9, np.int32)
    ome = np.zeros(9, np.int32)
    oa = np.zeros(1, np.int32)
    lib().ref_next(*a, int(action), op.ctypes.data_as(I32P), oe.ctypes.data_as(I32P), om.ctypes.data_as(I32P),
                   ome.ctypes.data_as(I32P), oa.ctypes.data_as(I32P))
    return (op.reshape(9, 9), oe.reshape(9, 9), om, ome, int(oa[0]))


def tensor(state):
    keep, a = _args(state)
    t = np.zeros(243, np.float32)
    lib().ref_tensor(*a, t.ctypes.data_as(F32P))
    return t


def to_string(state):
    keep, a = _args(state)
    buf = ctypes.create_string_buffer(4096)
    n = lib().ref_to_string(*a, buf, 4096)
    return buf.value.decode()


def search_hash(state, temperature, evaluate_count, batch_size):
    keep, a = _args(state)
    sc = np.zeros(81, np.float32)
    stats = np.zeros(3, np.int64)
    n = lib().ref_search_hash(*a, float(temperature), int(evaluate_count), int(batch_size),
                              sc.ctypes.data_as(F32P), stats.ctypes.data_as(I64P))
    return sc[:n].copy(), stats


def boltzman(xs, temperature):
    xs = np.ascontiguousarray(xs, np.float32)
    out = np.zeros_like(xs)
    lib().ref_boltzman(xs.ctypes.data_as(F32P), xs.size, float(temperature), out.ctypes.data_as(F32P))
    return out


def bench_tree(evaluate_count=50, batch_size=8, moves=200):
    sims = np.zeros(1, np.int64)
    rate = lib().ref_bench_tree(int(evaluate_count), int(batch_size), int(moves), sims.ctypes.data_as(I64P))
    return rate, int(sims[0])

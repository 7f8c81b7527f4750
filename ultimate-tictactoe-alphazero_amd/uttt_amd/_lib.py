"""ctypes binding of libuttt_engine.so (include/uttt_engine.h).

The library is built in-tree (``make -C ultimate-tictactoe-alphazero_amd``,
or ``__graft_entry__.build()``). There is no fallback: if it is missing,
importing the engine raises.
"""
import ctypes
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# UTTT_ENGINE_LIB: another in-tree build of the same C ABI (same-box A/B runs, tools/gpu_r3.sh abl)
LIB_PATH = os.environ.get("UTTT_ENGINE_LIB") or os.path.join(PKG_ROOT, "libuttt_engine.so")

UTTT_OK = 0
ERRORS = {-1: "UTTT_ERR_ARG", -2: "UTTT_ERR_HIP", -3: "UTTT_ERR_CAPACITY", -4: "UTTT_ERR_ORDER",
          -5: "UTTT_ERR_NODEVICE", -6: "UTTT_ERR_NONFINITE"}

KERNELS = {"select": 0, "apply": 1, "encode": 2, "scan": 3, "move_end": 4, "hash_eval": 5,
           # select latency counters (their value is in "bytes"; no launches)
           "select_levels": 6, "select_trees": 7, "select_max_levels_sum": 9,
           "select_trips": 10, "select_max_trips_sum": 12}


class UtttState(ctypes.Structure):
    """uttt_state_t: packed side-to-move-relative position (32 bytes)."""

    _fields_ = [("own", ctypes.c_uint32 * 3), ("opp", ctypes.c_uint32 * 3), ("mains", ctypes.c_uint32),
                ("active", ctypes.c_int32)]


STATE_DTYPE = np.dtype([("own", "<u4", (3,)), ("opp", "<u4", (3,)), ("mains", "<u4"), ("active", "<i4")])
assert STATE_DTYPE.itemsize == ctypes.sizeof(UtttState) == 32

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F32 = ctypes.c_float
_I32P = ctypes.POINTER(ctypes.c_int32)
_I64P = ctypes.POINTER(ctypes.c_int64)
_F32P = ctypes.POINTER(ctypes.c_float)
_F64P = ctypes.POINTER(ctypes.c_double)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_SP = ctypes.POINTER(UtttState)

# name -> (restype, argtypes)
SIGNATURES = {
    "uttt_last_error": (ctypes.c_char_p, []),
    "uttt_version": (ctypes.c_char_p, []),
    "uttt_state_initial": (None, [_SP]),
    "uttt_state_from_arrays": (ctypes.c_int, [_I32P, _I32P, _I32P, _I32P, _I32, _SP]),
    "uttt_state_to_arrays": (None, [_SP, _I32P, _I32P, _I32P, _I32P, _I32P]),
    "uttt_state_next": (ctypes.c_int, [_SP, _I32, _SP]),
    "uttt_state_legal_actions": (ctypes.c_int, [_SP, _I32P]),
    "uttt_state_is_lose": (ctypes.c_int, [_SP]),
    "uttt_state_is_draw": (ctypes.c_int, [_SP]),
    "uttt_state_is_done": (ctypes.c_int, [_SP]),
    "uttt_state_is_first_player": (ctypes.c_int, [_SP]),
    "uttt_state_input_hwc": (None, [_SP, _F32P]),
    "uttt_states_input_hwc": (ctypes.c_int, [_SP, _I64, _F32P]),
    "uttt_state_to_string": (ctypes.c_int, [_SP, ctypes.c_char_p, _I32]),
    "uttt_boltzman": (ctypes.c_int, [_F32P, _I32, _F32, _F32P]),
    "uttt_engine_create": (ctypes.c_int, [_I32, _I32, _I32, ctypes.POINTER(_P)]),
    "uttt_engine_destroy": (ctypes.c_int, [_P]),
    "uttt_engine_share_cache": (ctypes.c_int, [_P, _P]),
    "uttt_engine_own_stream": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_void_p)]),
    "uttt_engine_set_stream": (ctypes.c_int, [_P, _P]),
    "uttt_engine_device_bytes": (ctypes.c_int64, [_P]),
    "uttt_search_begin": (ctypes.c_int, [_P, _SP, _I32, _I32, _I32]),
    "uttt_search_begin_mode": (ctypes.c_int, [_P, _SP, _I32, _I32, _I32, _I32]),
    "uttt_search_select": (ctypes.c_int, [_P, _P, _I32P]),
    "uttt_search_select_async": (ctypes.c_int, [_P]),
    "uttt_selfplay_move_begin_async": (ctypes.c_int, [_P]),
    "uttt_selfplay_move_end_async": (ctypes.c_int, [_P]),
    "uttt_selfplay_move_result": (ctypes.c_int, [_P, _I64P, _I32P]),
    "uttt_search_count_copy": (ctypes.c_int, [_P, _P]),
    "uttt_search_select_async_to": (ctypes.c_int, [_P, ctypes.c_int32]),
    "uttt_search_select_async_tag": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32]),
    "uttt_search_count_ring": (ctypes.c_int, [_P, _P, _P]),
    "uttt_search_count_ptr": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_void_p)]),
    "uttt_search_pending": (ctypes.c_int, [_P, _SP, _I32P]),
    "uttt_search_apply": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _I32, _I32]),
    "uttt_eval_hash": (ctypes.c_int, [_P, _P, _I32, _P, _P]),
    "uttt_eval_hash_dev": (ctypes.c_int, [_P, _P, _P]),
    "uttt_round_hash_async": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "uttt_rounds_hash_async": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32]),
    "uttt_rounds_hash_move": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, _P, _P, _P]),
    "uttt_search_select_host": (ctypes.c_int, [_P, _P, _P, _P]),
    "uttt_search_apply_host": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, ctypes.c_int32]),
    "uttt_search_root_visits": (ctypes.c_int, [_P, _I32P, _I32P]),
    "uttt_search_scores": (ctypes.c_int, [_P, _F32, _F32P, _I32P]),
    "uttt_selfplay_begin": (ctypes.c_int, [_P, _I64, _I64, ctypes.c_uint32, _F32, _I32, _I32, _I64]),
    "uttt_selfplay_move_begin": (ctypes.c_int, [_P, _I32P]),
    "uttt_selfplay_move_end": (ctypes.c_int, [_P, _I64P]),
    "uttt_selfplay_get_rng": (ctypes.c_int, [_P, _I32, _U32P, _I32P]),
    "uttt_selfplay_set_rng": (ctypes.c_int, [_P, _I32, _U32P, _I32]),
    "uttt_selfplay_games": (ctypes.c_int, [_P, _I64P, _I64P, _I32P, _I64, _I64P]),
    "uttt_selfplay_plies": (ctypes.c_int, [_P, _SP, _F64P, ctypes.POINTER(ctypes.c_int8),
                                           ctypes.POINTER(ctypes.c_int8), _F32P, _I64, _I64P]),
    "uttt_engine_set_timing": (ctypes.c_int, [_P, _I32]),
    "uttt_engine_kernel_stats": (ctypes.c_int, [_P, _I32, ctypes.POINTER(ctypes.c_double), _I64P, _I64P]),
    "uttt_engine_reset_stats": (ctypes.c_int, [_P]),
    "uttt_engine_set_cache": (ctypes.c_int, [_P, _I32, _I32]),
    "uttt_engine_cache_clear": (ctypes.c_int, [_P]),
    "uttt_engine_cache_stats": (ctypes.c_int, [_P, _I64P, _I64P, _I64P]),
    "uttt_engine_cache_stats2": (ctypes.c_int, [_P, _I64P, _I64P, _I64P, _I64P]),
    "uttt_nn_stem": (ctypes.c_int, [_P, _P, _P, _P]),
    "uttt_nn_stem_states": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P]),
    "uttt_nn_heads": (ctypes.c_int, [_P, _P, _I32, _P, _P, _I32, _P]),
    "uttt_nn_heads_dev": (ctypes.c_int, [_P, _P, _P, _I32, _P, _P, _I32, _P]),
    "uttt_nn_wino3h_weights": (ctypes.c_int, [_F32P, _P, ctypes.POINTER(ctypes.c_float)]),
    "uttt_nn_conv3x3_wino3h": (ctypes.c_int, [_P, _P, ctypes.c_float, _P, _P, _P, _P, _I32, _P, _P, _I32, _I32, _P]),
    "uttt_nn_conv3x3_wino3h_dev": (ctypes.c_int, [_P, _P, ctypes.c_float, _P, _P, _P, _P, _I32, _P, _P, _I32, _P, _I32,
                                                  _P]),
    "uttt_nn_conv3x3_wino3h_f16": (ctypes.c_int, [_P, _P, ctypes.c_float, _P, _P, _P, _P, _I32, _P, _P, _I32, _I32,
                                                  _P]),
    "uttt_nn_conv3x3_wino3h_f16_dev": (ctypes.c_int, [_P, _P, ctypes.c_float, _P, _P, _P, _P, _I32, _P, _P, _I32, _P,
                                                      _I32, _P]),
    "uttt_nn_tower_wino3h_dev": (ctypes.c_int, [_P, _I64, _P, _P, _P, _I32, _P, _P, _I32, _P, _I32, _P, _I32, _P]),
    "uttt_nn_tower_ctl_words": (ctypes.c_int32, [_I32]),
    "uttt_nn_amax": (ctypes.c_int, [_P, _I64, _P, _P]),
    "uttt_nn_wino3h_set_split": (ctypes.c_int, [_I32]),
}

_lib = None


class EngineError(RuntimeError):
    pass


def load():
    """Load the engine library (torch first, so both share one HIP runtime)."""
    global _lib
    if _lib is None:
        import torch  # noqa: F401  (binds libamdhip64.so.7 before we do)
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C {PKG_ROOT}` (or __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


_diag = None


def load_diag():
    """The diagnostics library (libuttt_diag.so, `make -C <pkg> diag`): conv timing ablations and phase
    stamps for tools/diag. Never loaded by the product path or the tests."""
    global _diag
    if _diag is None:
        load()
        path = os.path.join(os.path.dirname(LIB_PATH), "libuttt_diag.so")
        if not os.path.exists(path):
            raise ImportError(f"{path} not built: run `make -C {PKG_ROOT} diag`")
        _diag = ctypes.CDLL(path)
    return _diag


def check(rc):
    if rc != UTTT_OK:
        msg = load().uttt_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(msg)
        raise EngineError(f"{ERRORS.get(rc, rc)}: {msg}")
    return rc


def ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))

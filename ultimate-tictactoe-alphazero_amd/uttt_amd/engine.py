"""Engine: Python handle on the C ABI (include/uttt_engine.h).

One ``Engine`` owns ``max_trees`` PUCT trees (or self-play slots) in HBM on one
GPU. All launches go to torch's current stream on that device, so the network
forward and the tree kernels are ordered without host synchronisation; the only
per-round sync is reading the number of pending leaves.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import STATE_DTYPE, UtttState, check, ptr


def as_states(states):
    """Sequence of uttt_cpp.State / packed bytes / STATE_DTYPE array -> STATE_DTYPE array."""
    if isinstance(states, np.ndarray) and states.dtype == STATE_DTYPE:
        return np.ascontiguousarray(states)
    out = np.zeros(len(states), STATE_DTYPE)
    for i, s in enumerate(states):
        raw = s.packed if hasattr(s, "packed") else bytes(s)
        out[i:i + 1] = np.frombuffer(raw, STATE_DTYPE)
    return out


def initial_states(n):
    out = np.zeros(n, STATE_DTYPE)
    out["active"] = -1
    return out


class RoundCount:
    """The pending-leaf count of a round enqueued with Engine.select_async: None until the
    host has read the copy back (SelfPlay fills it), then an int (int(rc) works from then on).
    Passed to a device-count evaluator in place of n."""
    __slots__ = ("n",)

    def __init__(self):
        self.n = None

    def __int__(self):
        if self.n is None:
            raise RuntimeError("round count not read back yet")
        return self.n

    __index__ = __int__


class Engine:
    def __init__(self, max_trees, max_sims=50, device=None):
        import torch

        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.EngineError("no ROCm GPU visible to torch; the engine runs only on MI355X (gfx950)")
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.max_trees = int(max_trees)
        self.max_sims = int(max_sims)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.lib.uttt_engine_create(self.device, self.max_trees, self.max_sims, ctypes.byref(h)))
        self.h = h
        self.n_trees = 0
        self.n_pending = 0
        self.use_stream()

    # -------------------------------------------------------------- plumbing --
    def use_stream(self, stream=None):
        """Launch on `stream` (default: torch's current stream on this device)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        check(self.lib.uttt_engine_set_stream(self.h, ctypes.c_void_p(s.cuda_stream)))
        self.stream = s

    def own_stream(self):
        """The engine's own non-blocking HIP stream as a torch ExternalStream."""
        import torch

        p = ctypes.c_void_p()
        check(self.lib.uttt_engine_own_stream(self.h, ctypes.byref(p)))
        return torch.cuda.ExternalStream(p.value, device=torch.device("cuda", self.device))

    def close(self):
        if getattr(self, "h", None):
            self.lib.uttt_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_bytes(self):
        return int(self.lib.uttt_engine_device_bytes(self.h))

    # ---------------------------------------------------------------- search --
    SEMANTICS = {"cpp": 0, "py": 1}

    def search_begin(self, roots, evaluate_count=50, batch_size=8, semantics="cpp"):
        """semantics "cpp": cpp/uttt_mcts.cpp (pv_mcts_cpp, self-play); "py": pv_mcts.py (arena)."""
        roots = as_states(roots)
        check(self.lib.uttt_search_begin_mode(self.h, roots.ctypes.data_as(ctypes.POINTER(UtttState)), len(roots),
                                              int(evaluate_count), int(batch_size), self.SEMANTICS[semantics]))
        self.n_trees = len(roots)

    def select(self, nn_input=None):
        """One round; writes NCHW inputs into nn_input (device tensor) and returns the pending count."""
        n = ctypes.c_int32()
        p = ctypes.c_void_p(nn_input.data_ptr()) if nn_input is not None else None
        check(self.lib.uttt_search_select(self.h, p, ctypes.byref(n)))
        self.n_pending = n.value
        return n.value

    def select_async(self):
        """One round with the pending count left on the device (uttt_search_select_async): the
        network's *_dev entry points and apply() read it there; count_copy() fetches it."""
        check(self.lib.uttt_search_select_async(self.h))
        self.n_pending = None

    def select_async_to(self, ring_slot):
        """select_async whose scan also writes the round's counts into slot ring_slot of the engine's
        host-visible ring (count_ring()): readable once an event recorded after it has completed."""
        check(self.lib.uttt_search_select_async_to(self.h, int(ring_slot)))
        self.n_pending = None

    def _next_tag(self):
        """The next ring tag, kept in the int32 range the C ABI takes (a wrapped ctypes value would never
        compare equal to the Python int the waiter holds)."""
        return (getattr(self, "tag", 0) + 1) & 0x7FFFFFFF

    def select_async_tag(self, ring_slot):
        """select_async_to whose scan stores a new tag into word 3 of the ring slot after the counts; returns
        the tag (the counts are readable once the slot's word 3 holds it)."""
        self.tag = self._next_tag()
        check(self.lib.uttt_search_select_async_tag(self.h, int(ring_slot), self.tag))
        self.n_pending = None
        return self.tag

    def count_ring(self):
        """The engine's host count ring as an (n_slots, 4) int32 numpy view of pinned host memory."""
        p, n = ctypes.c_void_p(), ctypes.c_int32()
        check(self.lib.uttt_search_count_ring(self.h, ctypes.byref(p), ctypes.byref(n)))
        arr = ctypes.cast(p, ctypes.POINTER(ctypes.c_int32 * (4 * n.value))).contents
        return np.frombuffer(arr, dtype=np.int32).reshape(n.value, 4)

    def count_copy(self, dst):
        """Enqueue a copy of the round's [pending, stopped, trees with simulations left after
        this round] counts into dst (pinned int32 host tensor of >= 3)."""
        check(self.lib.uttt_search_count_copy(self.h, ctypes.c_void_p(dst.data_ptr())))

    def count_ptr(self):
        """Device address of the round's counts (see count_copy)."""
        p = ctypes.c_void_p()
        check(self.lib.uttt_search_count_ptr(self.h, ctypes.byref(p)))
        return p

    def pending(self):
        n = self.n_pending
        st = np.zeros(n, STATE_DTYPE)
        k = np.zeros(n, np.int32)
        check(self.lib.uttt_search_pending(self.h, st.ctypes.data_as(ctypes.POINTER(UtttState)), ptr(k, ctypes.c_int32)))
        return st, k

    def apply(self, policy, value, per_copy=False):
        """policy: (rows, >=81) f32, value: (rows,) or (rows,1) f32 — device tensors or numpy arrays."""
        if isinstance(policy, np.ndarray):
            pol = np.ascontiguousarray(policy, np.float32)
            val = np.ascontiguousarray(value, np.float32).reshape(-1)
            check(self.lib.uttt_search_apply(self.h, ctypes.c_void_p(pol.ctypes.data), pol.shape[1],
                                             ctypes.c_void_p(val.ctypes.data), 1, int(per_copy), 0))
            return
        import torch

        assert policy.dtype == torch.float32 and value.dtype == torch.float32
        assert policy.is_cuda and value.is_cuda
        if policy.stride(1) != 1:
            policy = policy.contiguous()
        vld = value.stride(0)
        check(self.lib.uttt_search_apply(self.h, ctypes.c_void_p(policy.data_ptr()), policy.stride(0),
                                         ctypes.c_void_p(value.data_ptr()), vld, int(per_copy), 1))

    def eval_hash_dev(self, policy, value):
        """The hash evaluator on the round's pending leaves (states on the device, count on the
        device: rounds enqueued with select_async)."""
        check(self.lib.uttt_eval_hash_dev(self.h, ctypes.c_void_p(policy.data_ptr()),
                                          ctypes.c_void_p(value.data_ptr())))

    def rounds_hash_async(self, ring_slot, policy, value, n_rounds):
        """n_rounds consecutive hash rounds in one call (uttt_rounds_hash_async): ring slots ring_slot ..
        ring_slot + n_rounds - 1 (mod 8), tags tag + 1 .. tag + n_rounds; returns the last round's tag."""
        first = self._next_tag()
        self.tag = (first + n_rounds - 1) & 0x7FFFFFFF
        check(self.lib.uttt_rounds_hash_async(self.h, int(ring_slot), first, ctypes.c_void_p(policy.data_ptr()),
                                              ctypes.c_void_p(value.data_ptr()), int(n_rounds)))
        self.n_pending = None
        return self.tag

    def rounds_hash_move(self, ring_slot, policy, value, depth):
        """A move's whole hash-round loop in one call (uttt_rounds_hash_move): `depth` rounds in flight from ring
        slot ring_slot on, until a round leaves no tree with simulations. Returns (rounds enqueued, leaves,
        rounds with leaves); the rounds' ring slots and tags are consumed (self.tag is the last one)."""
        first = self._next_tag()
        nr, nl, nz = ctypes.c_int32(0), ctypes.c_int64(0), ctypes.c_int32(0)
        rc = self.lib.uttt_rounds_hash_move(self.h, int(ring_slot), first, ctypes.c_void_p(policy.data_ptr()),
                                            ctypes.c_void_p(value.data_ptr()), int(depth), ctypes.byref(nr),
                                            ctypes.byref(nl), ctypes.byref(nz))
        if nr.value:
            self.tag = (first + nr.value - 1) & 0x7FFFFFFF
        check(rc)
        self.n_pending = None
        return nr.value, nl.value, nz.value

    def round_hash_async(self, ring_slot, policy, value):
        """A whole round with the hash evaluator in one call (uttt_round_hash_async): select, scan (the counts
        and then a new tag into ring slot ring_slot), hash evaluation of the pending leaves, apply. Returns
        the tag; the round's counts in count_ring()[ring_slot] are valid once its word 3 equals it."""
        self.tag = self._next_tag()
        check(self.lib.uttt_round_hash_async(self.h, int(ring_slot), self.tag, ctypes.c_void_p(policy.data_ptr()),
                                             ctypes.c_void_p(value.data_ptr())))
        self.n_pending = None
        return self.tag

    def eval_hash(self, nn_input, n, policy, value):
        check(self.lib.uttt_eval_hash(self.h, ctypes.c_void_p(nn_input.data_ptr()), int(n),
                                      ctypes.c_void_p(policy.data_ptr()), ctypes.c_void_p(value.data_ptr())))

    def root_visits(self):
        v = np.zeros((self.n_trees, 81), np.int32)
        L = np.zeros(self.n_trees, np.int32)
        check(self.lib.uttt_search_root_visits(self.h, ptr(v, ctypes.c_int32), ptr(L, ctypes.c_int32)))
        return v, L

    def scores(self, temperature):
        s = np.zeros((self.n_trees, 81), np.float32)
        L = np.zeros(self.n_trees, np.int32)
        check(self.lib.uttt_search_scores(self.h, float(temperature), ptr(s, ctypes.c_float), ptr(L, ctypes.c_int32)))
        return s, L

    # ------------------------------------------------------------- self-play --
    def selfplay_begin(self, game_begin, game_end, seed_base, temperature=1.0, evaluate_count=50, batch_size=8,
                       arena_plies=None):
        if arena_plies is None:
            arena_plies = max(81, (game_end - game_begin) * 81)
        check(self.lib.uttt_selfplay_begin(self.h, int(game_begin), int(game_end), ctypes.c_uint32(seed_base),
                                           float(temperature), int(evaluate_count), int(batch_size),
                                           int(arena_plies)))
        self.n_trees = self.max_trees

    def move_begin(self):
        n = ctypes.c_int32()
        check(self.lib.uttt_selfplay_move_begin(self.h, ctypes.byref(n)))
        return n.value

    def move_end(self):
        n = ctypes.c_int64()
        check(self.lib.uttt_selfplay_move_end(self.h, ctypes.byref(n)))
        return n.value

    def move_begin_async(self):
        """Enqueue the next move's roots without reading the live count (move_result gives it)."""
        check(self.lib.uttt_selfplay_move_begin_async(self.h))

    def move_end_async(self):
        """Enqueue the move's end and a copy of its counters; read them with move_result once the
        stream has passed it."""
        check(self.lib.uttt_selfplay_move_end_async(self.h))

    def move_result(self):
        """(games finished so far, live slots of the next move) of the last move_end_async."""
        f, n = ctypes.c_int64(), ctypes.c_int32()
        check(self.lib.uttt_selfplay_move_result(self.h, ctypes.byref(f), ctypes.byref(n)))
        return f.value, n.value

    def get_rng(self, slot=0):
        key = np.zeros(624, np.uint32)
        pos = ctypes.c_int32()
        check(self.lib.uttt_selfplay_get_rng(self.h, int(slot), ptr(key, ctypes.c_uint32), ctypes.byref(pos)))
        return key, pos.value

    def set_rng(self, key, pos, slot=0):
        key = np.ascontiguousarray(key, np.uint32)
        check(self.lib.uttt_selfplay_set_rng(self.h, int(slot), ptr(key, ctypes.c_uint32), int(pos)))

    def games(self):
        n = ctypes.c_int64()
        check(self.lib.uttt_selfplay_games(self.h, None, None, None, 0, ctypes.byref(n)))
        ids = np.zeros(n.value, np.int64)
        off = np.zeros(n.value, np.int64)
        ln = np.zeros(n.value, np.int32)
        check(self.lib.uttt_selfplay_games(self.h, ptr(ids, ctypes.c_int64), ptr(off, ctypes.c_int64),
                                           ptr(ln, ctypes.c_int32), n.value, ctypes.byref(n)))
        return ids, off, ln

    def plies(self, with_inputs=True):
        n = ctypes.c_int64()
        check(self.lib.uttt_selfplay_plies(self.h, None, None, None, None, None, 0, ctypes.byref(n)))
        m = n.value
        st = np.zeros(m, STATE_DTYPE)
        pol = np.zeros((m, 81), np.float64)
        act = np.zeros(m, np.int8)
        val = np.zeros(m, np.int8)
        hwc = np.zeros((m, 243), np.float32) if with_inputs else None
        check(self.lib.uttt_selfplay_plies(
            self.h, st.ctypes.data_as(ctypes.POINTER(UtttState)), ptr(pol, ctypes.c_double), ptr(act, ctypes.c_int8),
            ptr(val, ctypes.c_int8), ptr(hwc, ctypes.c_float) if hwc is not None else None, m, ctypes.byref(n)))
        return {"states": st, "policies": pol, "actions": act, "values": val, "inputs_hwc": hwc}

    # ------------------------------------------------------- evaluation cache --
    def set_cache(self, log2_capacity=21, clear_every_moves=32):
        """Position -> evaluation table in HBM (0 = off). Exact for a deterministic evaluator."""
        check(self.lib.uttt_engine_set_cache(self.h, int(log2_capacity), int(clear_every_moves)))

    def share_cache(self, owner):
        """Use owner's evaluation table (engines on the same GPU); owner must outlive self."""
        check(self.lib.uttt_engine_share_cache(self.h, owner.h))
        self._cache_owner = owner  # keep the table's owner alive

    def cache_clear(self):
        check(self.lib.uttt_engine_cache_clear(self.h))

    def cache_stats(self):
        h, m, i, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.uttt_engine_cache_stats2(self.h, ctypes.byref(h), ctypes.byref(m), ctypes.byref(i),
                                                ctypes.byref(r)))
        return {"hits": h.value, "misses": m.value, "inserts": i.value, "replacements": r.value}

    # ------------------------------------------------------------- telemetry --
    def set_timing(self, on=True):
        check(self.lib.uttt_engine_set_timing(self.h, int(bool(on))))

    def reset_stats(self):
        check(self.lib.uttt_engine_reset_stats(self.h))

    def kernel_stats(self, name):
        ms = ctypes.c_double()
        ln = ctypes.c_int64()
        by = ctypes.c_int64()
        check(self.lib.uttt_engine_kernel_stats(self.h, _lib.KERNELS[name], ctypes.byref(ms), ctypes.byref(ln),
                                                ctypes.byref(by)))
        return {"ms": ms.value, "launches": ln.value, "bytes": by.value}

#!/usr/bin/env python3
"""Where a k_select dependent round trip goes: the tree-only configuration (hash
evaluator, 4,096 trees, 50 sims, B = 8, one lane) on the diagnostics engine build
(libuttt_engine_diag.so: k_select's SelClock phase marks compiled in; loaded through UTTT_ENGINE_LIB),
aged like the bench, then the phase cycles of the timed moves: per launch, summed over trees and per
tree, for all trees and for the heavy trees (>= 24 round trips in the launch, the ones that set a
launch's length). Each mark drains the wave's memory counters, so the phases do not overlap (the
instrumented launch is slower than the product's). One JSON line.
usage: python tools/diag/select_cycles.py [age] [moves] [pretouch 0-3 (engine.hip g_sel_pretouch)]"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")
os.environ["UTTT_ENGINE_LIB"] = os.path.join(PKG, "libuttt_engine_diag.so")
sys.path[:0] = [PKG]

import torch  # noqa: E402
from uttt_amd import SelfPlay, _lib  # noqa: E402

PHASES = ["root", "group_loads", "puct", "argmax", "next_state", "leaf_checks", "terminal_backup", "cache_probe",
          "hit_expand", "hit_tail", "queue", "root_state"]


def main():
    age = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    moves = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    lib = _lib.load()
    fn = lib.uttt_diag_select_cycles
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    fn.restype = ctypes.c_int
    n = 2 * len(PHASES) + 2
    buf = (ctypes.c_ulonglong * n)()
    pretouch = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if pretouch:
        pt = lib.uttt_diag_select_pretouch
        pt.argtypes = [ctypes.c_int32]
        pt.restype = ctypes.c_int
        assert pt(pretouch) == 0
    sp = SelfPlay(4096, 50, 8, 1.0, lanes=1, cache_log2=23)
    sp.begin(0, 4096 * (age + moves + 4), 1234, arena_plies=4096 * (age + moves + 4))
    sp.steps(age)
    torch.cuda.synchronize()
    sp.reset_stats()
    sp.set_timing(True)
    fn(None, 1)
    sp.steps(moves)
    torch.cuda.synchronize()
    assert fn(buf, 0) == 0
    v = list(buf)
    st = sp.kernel_stats("select")
    trips = sp.kernel_stats("select_trips")["bytes"]
    launches = max(st["launches"], 1)
    trees_all, trees_heavy = v[2 * len(PHASES)], v[2 * len(PHASES) + 1]
    out = {"config": "tree-only 4096 x 50, B 8, hash evaluator, 1 lane, diagnostics engine build", "age": age,
           "pretouch": pretouch,
           "moves": moves, "select_launches": st["launches"], "select_us_per_launch_instrumented":
           round(st["ms"] * 1e3 / launches, 2), "trips_per_tree_per_launch": round(trips / max(trees_all, 1), 2),
           "trees_per_launch": round(trees_all / launches, 1), "heavy_trees_per_launch": round(trees_heavy / launches, 1),
           "cycles_per_tree": {p: round(v[i] / max(trees_all, 1), 1) for i, p in enumerate(PHASES)},
           "cycles_per_heavy_tree": {p: round(v[len(PHASES) + i] / max(trees_heavy, 1), 1)
                                     for i, p in enumerate(PHASES)}}
    out["cycles_per_tree"]["total"] = round(sum(v[:len(PHASES)]) / max(trees_all, 1), 1)
    out["cycles_per_heavy_tree"]["total"] = round(sum(v[len(PHASES):2 * len(PHASES)]) / max(trees_heavy, 1), 1)
    # the last launch's wall clock per tree (s_memrealtime, 100 MHz: 10 ns ticks), live trees only
    rtf = lib.uttt_diag_select_rt
    rtf.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    rtf.restype = ctypes.c_int
    rb = (ctypes.c_ulonglong * (4 * 4096))()
    assert rtf(rb, 4096) == 0
    import numpy as np
    r = np.frombuffer(rb, dtype=np.uint64).reshape(4096, 4).astype(np.int64)
    live = r[:, 1] > 0
    if live.any():
        t0 = r[:, 0].min()
        q = lambda x: [round(float(v) / 100.0, 2) for v in np.percentile(x, [0, 10, 50, 90, 100])]
        out["last_launch_us"] = {
            "percentiles": [0, 10, 50, 90, 100], "live_trees": int(live.sum()),
            "start_after_first_start": q(r[:, 0] - t0),
            "first_root_phase": q(r[live, 1] - r[live, 0]),
            "end_after_first_start": q(r[:, 2] - t0),
            "wave_duration": q(r[:, 2] - r[:, 0]),
            "trips": [int(v) for v in np.percentile(r[:, 3], [0, 10, 50, 90, 100])]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where Option A's module time goes: uttt_cpp.pv_mcts_scores with a
model that returns fixed arrays (no device work), on the 40 positions of tools/diag/latency_single.py, and
the resident wave's own time split per search (uttt_search1_time_split: descents, applies, waits for the
host). The host's share is the wall time minus the wave's busy time. One JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402


def main():
    import uttt_cpp
    import _uttt_cpp
    rng = np.random.RandomState(0)
    states = []
    s = uttt_cpp.State()
    while not s.is_done() and len(states) < 40:
        states.append(s)
        s = s.next(int(rng.choice(s.legal_actions())))
    fixed_p, fixed_v = np.full(81, 1.0 / 81, np.float32), 0.0
    calls = {"n": 0, "s": 0.0}

    def fixed(sl):
        t0 = time.perf_counter()
        r = [(fixed_p, fixed_v)] * len(sl)
        calls["n"] += 1
        calls["s"] += time.perf_counter() - t0
        return r

    out = {"metric": "resident one-tree search: time split per search (ms), fixed-array model"}
    for name, kw in (("copies", {}), ("dedup", {"dedup": True})):
        for st in states[:3]:
            uttt_cpp.pv_mcts_scores(model=fixed, state=st, temperature=1.0, evaluate_count=50, batch_size=8, **kw)
        reps = 5
        wall, split = 0.0, np.zeros(3)
        calls.update(n=0, s=0.0)
        for _ in range(reps):
            for st in states:
                t = time.perf_counter()
                uttt_cpp.pv_mcts_scores(model=fixed, state=st, temperature=1.0, evaluate_count=50, batch_size=8, **kw)
                wall += time.perf_counter() - t
                split += np.asarray(_uttt_cpp._search1_time_split())
        n = reps * len(states)
        out[name] = {"wall_ms": round(wall * 1e3 / n, 4), "select_ms": round(split[0] / n, 4),
                     "apply_ms": round(split[1] / n, 4), "wait_ms": round(split[2] / n, 4),
                     "flushes": round(calls["n"] / n, 2), "model_ms": round(calls["s"] * 1e3 / n, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

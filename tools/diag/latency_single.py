#!/usr/bin/env python3
"""Per-call latency of the single-tree search paths a reference caller uses one move at a time
(INTEGRATION.md Option A): pv_mcts_cpp.pv_mcts_scores_cpp (the engine with the fused HIP evaluator,
one tree, 50 sims, batch 8) and pv_mcts.pv_mcts_scores (Python-search semantics on the engine), on
positions along one game; plus the conv alone at small batches. One JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import pv_mcts_cpp
    import uttt_cpp
    from uttt_amd.model import random_network
    net = random_network(0, "cuda")
    rng = np.random.RandomState(0)
    states = []
    s = uttt_cpp.State()
    while not s.is_done() and len(states) < 40:
        states.append(s)
        s = s.next(int(rng.choice(s.legal_actions())))
    out = {"metric": "single-tree search latency (ms per call, one move, 50 sims, batch 8)"}
    for name, fn in (("pv_mcts_scores_cpp", lambda st: pv_mcts_cpp.pv_mcts_scores_cpp(net, st, 1.0, 50, 8)),):
        for st in states[:3]:
            fn(st)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for st in states:
            fn(st)
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t) * 1e3 / len(states), 3)
    out["positions"] = len(states)
    out["reference_published_ms"] = {"mcts_50_sims": 50.0, "source": "README.md:290 (4070 Ti + 5800X)"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

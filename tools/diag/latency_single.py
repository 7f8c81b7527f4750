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
    # Option A: the reference's pv_mcts_cpp / self_play_cpp drivers unchanged over this
    # uttt_cpp. "torch": the reference's own flush glue (pv_mcts_cpp.py:37-87: to_input_tensor per state, NCHW
    # torch tensor, model(x), .cpu()) with the PyTorch DualNetwork; "fused": this build's pv_mcts_cpp, whose
    # callback hands the states to the fused HIP evaluator instead.
    for name, kind in (("pv_mcts_scores_cpp_fused", "auto"), ("pv_mcts_scores_cpp_torch", "torch")):
        os.environ["UTTT_EVALUATOR"] = kind
        fn = lambda st: pv_mcts_cpp.pv_mcts_scores_cpp(net, st, 1.0, 50, 8)  # noqa: E731
        for st in states[:3]:
            fn(st)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for st in states:
            fn(st)
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t) * 1e3 / len(states), 3)
    os.environ.pop("UTTT_EVALUATOR")
    out["positions"] = len(states)
    # self_play_cpp.self_play's 500 games one move at a time: 26,651 plies in the build's 500-game cycle
    # (profiles/r3/cycle_fp32_final.json), i.e. 53.3 moves per game
    plies = 26651
    out["projected_500_games_s"] = {k: round(out[k] * plies / 1e3, 1) for k in
                                    ("pv_mcts_scores_cpp_fused", "pv_mcts_scores_cpp_torch")}
    out["projected_sims_per_s"] = {k: round(50 * 1e3 / out[k], 1) for k in
                                   ("pv_mcts_scores_cpp_fused", "pv_mcts_scores_cpp_torch")}
    out["reference_published_ms"] = {"mcts_50_sims": 50.0, "source": "README.md:290 (4070 Ti + 5800X)"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

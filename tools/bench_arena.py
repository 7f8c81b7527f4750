#!/usr/bin/env python3
"""Arena-path throughput: evaluate_network / self_play.py semantics
(UTTT_SEMANTICS_PY) with two random DualNetworks (seeds 0 and 1) on the fused HIP evaluator,
all games concurrent. Prints one JSON line. CPU baseline ("port"): the oracle's restatement
of pv_mcts.py with the same DualNetwork on the host (torch CPU threads), bounded sample.

usage: python tools/bench_arena.py [--games 1024] [--mode arena|selfplay] [--cpu-seconds 10]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]


def cpu_baseline(seconds):
    import numpy as np
    import torch
    from oracle import core
    from uttt_amd.model import random_network
    net = random_network(0).eval()
    threads = torch.get_num_threads()

    last = {}

    def ev(x):  # a flush's copies are one state: one network call per flush, like predict_batch's one call
        key = np.asarray(x, np.float32).tobytes()
        if key not in last:
            with torch.no_grad():
                p, v = net(torch.from_numpy(np.asarray(x, np.float32).reshape(1, 3, 9, 9)))
            last.clear()
            last[key] = (p[0].numpy(), float(v[0, 0]))
        return last[key]

    s = core.OrState.initial()
    sims, t0, moves = 0, time.perf_counter(), 0
    rng = np.random.RandomState(0)
    while time.perf_counter() - t0 < seconds:
        if s.is_done():
            s = core.OrState.initial()
        core.pv_mcts_scores_py_callback(s, 1.0, 50, 8, ev)
        sims += 50
        moves += 1
        legal = s.legal_actions()
        s = s.next(int(legal[rng.randint(len(legal))]))
    dt = time.perf_counter() - t0
    return {"value": sims / dt, "unit": "simulations/s", "cores": threads, "kind": "port",
            "sample": f"{moves} pv_mcts.py searches (50 sims, batch 8) by the oracle restatement with a CPU "
                      f"DualNetwork (one network call per flush), {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=1024)
    ap.add_argument("--mode", choices=["arena", "selfplay"], default="arena")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    import torch
    from uttt_amd import arena
    from uttt_amd.model import random_network
    from uttt_amd.nnfast import FusedNetworkEvaluator
    dev = torch.device("cuda", 0)
    nets = [random_network(0, dev), random_network(1, dev)]
    mk = lambda m, e: FusedNetworkEvaluator(m, e)  # noqa: E731
    G = args.games
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.mode == "arena":
        avg, points, actions = arena.evaluate_network(nets[0], nets[1], G, 1.0, 777, make_evaluator=mk)
        moves = sum(len(a) for a in actions)
    else:
        games = arena.self_play_py(nets[0], G, 777, make_evaluator=mk)
        moves = sum(len(g) for g in games)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"metric": f"pv_mcts.py-semantics simulations/s ({args.mode}, {G} concurrent games, 50 sims/move, "
                     f"batch 8)", "value": moves * 50 / dt, "unit": "simulations/s", "games": G, "moves": moves,
           "seconds": round(dt, 3), "dtype": "f32", "data": "synthetic: random-init DualNetworks (seeds 0, 1)"}
    if args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

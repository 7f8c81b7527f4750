#!/usr/bin/env python3
"""How many of a round's network rows are the same position as another row of that round (the
evaluation cache only answers a position from the next round on)? Headline shape (4,096 games x 50
sims, B 8, one lane, cache 2^23), the fused network as the evaluator, blocking rounds so the host sees
each round's NCHW rows; aged like the bench. One JSON line.
usage: python tools/diag/round_duplicates.py [age] [moves]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]
os.environ["UTTT_ASYNC_ROUNDS"] = "0"

import torch  # noqa: E402
from uttt_amd import SelfPlay  # noqa: E402
from uttt_amd.model import random_network  # noqa: E402
from uttt_amd.nnfast import FusedNetworkEvaluator  # noqa: E402


def main():
    age = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    moves = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    net = random_network(0, "cuda")
    stats = {"rows": 0, "unique": 0, "rounds": 0}
    counting = [False]

    def make(eng):
        fe = FusedNetworkEvaluator(net, eng)

        def ev(x, n):
            if counting[0] and n:
                rows = x[:int(n)].reshape(int(n), -1)
                # the 243 inputs are 0/1: pack to bytes and count distinct rows
                packed = (rows > 0.5).to(torch.uint8)
                u = torch.unique(packed, dim=0).shape[0]
                stats["rows"] += int(n)
                stats["unique"] += int(u)
                stats["rounds"] += 1
            return fe(x, n)

        ev.needs_input = True
        ev.device_count = False
        return ev

    sp = SelfPlay(4096, 50, 8, 1.0, lanes=1, cache_log2=23)
    sp.set_evaluator(make)
    sp.begin(0, 4096 * (age + moves + 4), 1234, arena_plies=4096 * (age + moves + 4))
    sp.steps(age)
    counting[0] = True
    sp.steps(moves)
    torch.cuda.synchronize()
    stats["duplicate_share"] = round(1.0 - stats["unique"] / max(stats["rows"], 1), 4)
    stats.update({"age": age, "moves": moves, "cache": sp.cache_stats()})
    print(json.dumps(stats), flush=True)


if __name__ == "__main__":
    main()

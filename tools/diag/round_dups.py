#!/usr/bin/env python3
"""How many of a round's network rows are the same position (bench shape: 4,096 games x 50 sims, batch 8,
evaluation cache 2^23, games aged as the bench ages them). The cache removes repeats across rounds; this
counts repeats WITHIN a round (several trees queueing one position before any of them is evaluated), the
rows a within-round dedup would save. Plain PyTorch evaluator on the folded net (rows counted, not timed).
One JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import torch  # noqa: E402


def main():
    from uttt_amd import SelfPlay
    from uttt_amd.model import FoldedDualNetwork, random_network
    games = int(os.environ.get("GAMES", 4096))
    age = int(os.environ.get("AGE", 60))
    steps = int(os.environ.get("STEPS", 20))
    net = FoldedDualNetwork(random_network(0, "cuda")).cuda()
    stats = {"calls": 0, "rows": 0, "unique": 0}
    counting = [False]

    def make(eng):
        @torch.no_grad()
        def ev(x, n):
            if counting[0] and n > 0:
                flat = x[:n].reshape(n, -1).to(torch.uint8)
                stats["calls"] += 1
                stats["rows"] += n
                stats["unique"] += int(torch.unique(flat, dim=0).shape[0])
            p, v = net(x[:n])
            return p.float(), v.float()
        ev.needs_input = True
        ev.device_count = False
        return ev

    sp = SelfPlay(games, 50, 8, 1.0, device=0, cache_log2=23, lanes=1)
    sp.set_evaluator(make)
    sp.begin(0, (age + steps + 2) * games, 1234, arena_plies=(age + steps + 2) * games)
    for i in range(0, age, 10):
        sp.steps(min(10, age - i))
        print(f"aged {i + 10}", flush=True)
    counting[0] = True
    sp.steps(steps)
    torch.cuda.synchronize()
    out = {"metric": "within-round duplicate network rows (bench shape)", "games": games, "age": age,
           "steps": steps, **stats, "dup_frac": round(1 - stats["unique"] / max(stats["rows"], 1), 4),
           "cache": sp.cache_stats()}
    print(json.dumps(out, default=str))


if __name__ == "__main__":
    main()

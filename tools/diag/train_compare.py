#!/usr/bin/env python3
"""Loss curves of the training paths on the same real history: 500 self-play games of the seed-0
DualNetwork on the engine (the cycle's first self-play), then EPOCHS epochs from the same weights
with (a) the eager loop (the reference's own form), (b) the fp32 HIP-graph step, (c) the f16 graph
step. Prints per-epoch mean losses and the time per epoch."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import torch  # noqa: E402
from uttt_amd import SelfPlay, history_from_records, train  # noqa: E402
from uttt_amd.model import random_network  # noqa: E402


def main():
    epochs = int(os.environ.get("EPOCHS", "12"))
    dev = torch.device("cuda", 0)
    net = random_network(0, dev)
    sp = SelfPlay(500, 50, 8, 1.0, device=0, model=net)
    sp.run(0, 500, 1234)
    hist = history_from_records(sp.records())
    print(f"history: {len(hist)} plies", flush=True)
    for name, kw in (("eager_fp32", dict(graph=False)), ("graph_fp32", dict(graph=True)),
                     ("graph_f16", dict(graph=True, precision="f16")), ("eager_fp32_again", dict(graph=False))):
        m = random_network(0, dev).train()
        torch.cuda.synchronize()
        t = time.perf_counter()
        losses = train.train_network(m, hist, epochs=epochs, device=dev, log=None, **kw)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(name, f"{dt / epochs:.3f} s/epoch", [round(x, 4) for x in losses], flush=True)


if __name__ == "__main__":
    main()

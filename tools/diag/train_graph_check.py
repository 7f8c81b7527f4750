#!/usr/bin/env python3
"""One optimiser step of the eager loop and of the HIP-graph step (uttt_amd.train.GraphedStep) from the
same weights on the same batch: parameter deltas and losses side by side, then a few steps each."""
import copy
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from uttt_amd import train  # noqa: E402
from uttt_amd.model import random_network  # noqa: E402


def main():
    torch.backends.cudnn.benchmark = bool(int(os.environ.get("BENCH", "0")))
    dev = torch.device("cuda", 0)
    rng = np.random.RandomState(0)
    n = 1024
    xs = (rng.rand(n, 9, 9, 3) < 0.3).astype(np.float32)
    ps = rng.rand(n, 81)
    ps /= ps.sum(axis=1, keepdims=True)
    vs = rng.randint(-1, 2, size=n)
    hist = [[xs[i], ps[i], int(vs[i])] for i in range(n)]
    x, p, v = (torch.from_numpy(a).to(dev) for a in train.history_arrays(hist))
    idx = torch.arange(128, device=dev)
    for steps in (1, 5):
        m_e = random_network(0).to(dev).train()
        m_g = copy.deepcopy(m_e)
        w0 = {k: t.detach().clone() for k, t in m_e.state_dict().items()}
        opt_e = torch.optim.Adam(m_e.parameters(), lr=1e-3)
        le = [float(train.train_step(m_e, opt_e, x[idx], p[idx], v[idx])) for _ in range(steps)]
        lr_t = torch.tensor(1e-3, device=dev)
        opt_g = torch.optim.Adam(m_g.parameters(), lr=lr_t, capturable=True, foreach=True)
        gs = train.GraphedStep(m_g, opt_g, x, p, v, 128)
        after_capture = max(float((t - w0[k]).abs().max()) for k, t in m_g.state_dict().items() if t.is_floating_point())
        lg = []
        for _ in range(steps):
            gs.loss_sum.zero_()
            gs.step(idx)
            torch.cuda.synchronize()
            lg.append(float(gs.loss_sum))
        de = {k: float((t - w0[k]).abs().max()) for k, t in m_e.state_dict().items() if t.is_floating_point()}
        dg = {k: float((t - w0[k]).abs().max()) for k, t in m_g.state_dict().items() if t.is_floating_point()}
        diff = {k: float((m_e.state_dict()[k] - m_g.state_dict()[k]).abs().max()) for k in de}
        worst = sorted(diff.items(), key=lambda kv: -kv[1])[:5]
        print(f"steps {steps}: eager losses {le} graph losses {lg}; weights moved by capture+restore {after_capture:.3g}; "
              f"max |delta| eager {max(de.values()):.3g} graph {max(dg.values()):.3g}; worst eager-graph {worst}",
              flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A few product launches of the tower conv (uttt_nn_conv3x3_wino3h, and the f16 mode's
uttt_nn_conv3x3_wino3h_f16) at N boards, plain form, for counter passes: each precision's kernel
has its own name in the trace (the MODE template bit), so one process covers both.
usage: python tools/diag/conv_once.py N [reps] [precisions, default f32,f16]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import torch  # noqa: E402
from uttt_amd.model import fold_bn, random_network  # noqa: E402
from uttt_amd.nnfast import board_amax, conv3x3_wino3h, wino3h_weights  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    precs = (sys.argv[3] if len(sys.argv) > 3 else "f32,f16").split(",")
    net = random_network(0)
    w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
    u, su = wino3h_weights(w)
    u, b = u.cuda(), b.cuda()
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
    xa = board_amax(x)
    for p in precs:
        for _ in range(reps):
            y = conv3x3_wino3h(x, u, su, b, x_amax=xa, precision=p)
        torch.cuda.synchronize()
        print(p, n, float(y.abs().sum()), flush=True)


if __name__ == "__main__":
    main()

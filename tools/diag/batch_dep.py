"""Diagnostic: does k_wino3h_conv's output for a board depend on its position in the batch?
Prints, per offset, the boards/tiles whose output bits differ from the offset-0 run."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]
from uttt_amd.model import fold_bn, random_network  # noqa: E402
from uttt_amd.nnfast import conv3x3_wino3h, wino3h_weights  # noqa: E402

net = random_network(3)
w, b = fold_bn(net.residual_blocks[4].conv2, net.residual_blocks[4].bn2)
u, su = wino3h_weights(w)
u, b = u.cuda(), b.cuda()
g = torch.Generator().manual_seed(4)
x = torch.relu(torch.randn(14, 81, 128, generator=g)).cuda()
for res in (False, True):
    r = torch.randn(14, 81, 128, generator=g).cuda() if res else None
    y0 = conv3x3_wino3h(x, u, su, b, r)
    for off in range(1, 8):
        xb = torch.zeros(14 + off, 81, 128, device="cuda")
        xb[off:] = x
        rb = None
        if res:
            rb = torch.zeros(14 + off, 81, 128, device="cuda")
            rb[off:] = r
        yb = conv3x3_wino3h(xb, u, su, b, rb)[off:]
        d = (yb != y0).reshape(14, 9, 9, 128)
        bad = []
        for bi in range(14):
            if d[bi].any():
                pos = d[bi].any(dim=2).nonzero().tolist()
                tiles = sorted({(p[0] // 3) * 3 + p[1] // 3 for p in pos})
                bad.append((bi, (bi + off) % 7, tiles, (yb[bi] - y0[bi]).abs().max().item()))
        print("res", res, "off", off, "bad boards (board, group pos, tiles, maxdiff):", bad)

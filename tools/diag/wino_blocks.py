"""Diagnostic: per-block error of the Winograd conv chain vs a float64 torch chain."""
import sys
import numpy as np
import torch
import torch.nn.functional as F
sys.path[:0] = ['.', 'ultimate-tictactoe-alphazero_amd']
from uttt_amd.model import fold_bn, random_network
from uttt_amd.nnfast import conv3x3_wino, wino_weights

net = random_network(0)
g = torch.Generator().manual_seed(0)
n = 300
x = torch.relu(torch.randn(n, 81, 128, generator=g)).cuda()
xr = x.double()
for i, b in enumerate(net.residual_blocks):
    w1, b1 = fold_bn(b.conv1, b.bn1)
    w2, b2 = fold_bn(b.conv2, b.bn2)
    u1, u2 = wino_weights(w1).cuda(), wino_weights(w2).cuda()
    w1, b1, w2, b2 = w1.cuda(), b1.cuda(), w2.cuda(), b2.cuda()
    t = conv3x3_wino(x, u1, b1)
    y = conv3x3_wino(t, u2, b2, x)

    def ref(a, w, bb):
        an = a.reshape(n, 9, 9, 128).permute(0, 3, 1, 2)
        return F.conv2d(an, w.double(), bb.double(), padding=1).permute(0, 2, 3, 1).reshape(n, 81, 128)

    # one-step reference from the kernel's own input (isolates this block's error)
    t1 = torch.relu(ref(x.double(), w1, b1))
    y1 = torch.relu(ref(t.double(), w2, b2) + x.double())
    e_t = ((t.double() - t1).abs().max() / t1.abs().max()).item()
    e_y = ((y.double() - y1).abs().max() / y1.abs().max()).item()
    # chain reference
    tr = torch.relu(ref(xr, w1, b1))
    xr = torch.relu(ref(tr, w2, b2) + xr)
    e_chain = ((y.double() - xr).abs().max() / xr.abs().max()).item()
    bad = ((y.double() - y1).abs() > 1e-3 * y1.abs().max()).nonzero()
    print(f"block {i}: step-rel-err conv1 {e_t:.2e} conv2 {e_y:.2e}; chain {e_chain:.2e}; max|y| {y.abs().max().item():.3e}; "
          f"bad elems {len(bad)} rows {sorted(set(bad[:, 0].tolist()))[:10]} pos {sorted(set(bad[:, 1].tolist()))[:10]} ch {sorted(set(bad[:, 2].tolist()))[:10]}", flush=True)
    x = y

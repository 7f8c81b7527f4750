"""Isolated timing of the tower conv at small batches: the persistent kernel (split 1) against the
channel-split kernel k_wino3s_conv (split 2; splits 4 and 8 were measured slower at every size and are
in the diagnostics library only, tools/diag/conv_small_pf.py), plain and residual forms, one launch at a time
(HIP events around 20 launches on the current stream), and a bit comparison of every split's outputs
with the persistent kernel's. usage: conv_split_time.py [boards ...]"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]
from uttt_amd.model import fold_bn, random_network  # noqa: E402
from uttt_amd.nnfast import board_amax, conv3x3_wino3h, set_conv_split, wino3h_weights  # noqa: E402


def main():
    boards = [int(a) for a in sys.argv[1:]] or [1, 4, 8, 16, 25, 50, 100, 250, 500, 1000]
    net = random_network(0)
    w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
    u, su = wino3h_weights(w)
    u, b = u.cuda(), b.cuda()
    g = torch.Generator().manual_seed(1)
    rows = []
    for n in boards:
        x = torch.relu(torch.randn(n, 81, 128, generator=g)).cuda()
        r = torch.randn(n, 81, 128, generator=g).cuda()
        xa = board_amax(x)
        row = {"boards": n}
        ref = {}
        for split in (1, 2):
            set_conv_split(split)
            outs = {}
            for res in (False, True):
                ya = torch.zeros(n, dtype=torch.int32, device="cuda")
                y = conv3x3_wino3h(x, u, su, b, r if res else None, y_amax=ya)
                outs[res] = (y, ya)
                if split == 1:
                    ref[res] = (y, ya)
                else:
                    same = torch.equal(y, ref[res][0]) and torch.equal(ya, ref[res][1])
                    row.setdefault("bits_equal", True)
                    row["bits_equal"] = row["bits_equal"] and same
            times = []
            for rep in range(3):
                for res in (False, True):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(20):
                        conv3x3_wino3h(x, u, su, b, r if res else None, x_amax=xa)
                    e1.record()
                    torch.cuda.synchronize()
                    times.append((res, e0.elapsed_time(e1) * 1e3 / 20))
            row[f"split{split}_plain_us"] = round(min(t for rr, t in times if not rr), 1)
            row[f"split{split}_res_us"] = round(min(t for rr, t in times if rr), 1)
        set_conv_split(-1)
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

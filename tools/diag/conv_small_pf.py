"""Small-batch conv latency against prefetch depth (diagnostic): the product path (persistent
kernel, or the split-2 kernel it picks for <= 16 boards) against k_wino3s_conv at split 2 / 4 and
U prefetch 3 / 6 / 9 / 12 points (libuttt_diag.so), HIP events around 20 launches, min of 3, plain and
residual forms; outputs compared bit for bit with the persistent kernel.
usage: conv_small_pf.py [boards ...]"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]
from uttt_amd import _lib  # noqa: E402
from uttt_amd.model import fold_bn, random_network  # noqa: E402
from uttt_amd.nnfast import board_amax, conv3x3_wino3h, set_conv_split, wino3h_weights  # noqa: E402


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timeit(fn):
    best = 1e30
    for _ in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
    return round(best, 1)


def main():
    boards = [int(a) for a in sys.argv[1:]] or [1, 4, 8, 16, 25, 50]
    dl = _lib.load_diag()
    dl.uttt_diag_wino3s.restype = ctypes.c_int
    at = [ctypes.c_void_p] * 7 + [ctypes.c_int32] * 3 + [ctypes.c_void_p]
    at[2] = ctypes.c_float
    dl.uttt_diag_wino3s.argtypes = at
    net = random_network(0)
    w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
    u, su = wino3h_weights(w)
    u, b = u.cuda(), b.cuda()
    g = torch.Generator().manual_seed(1)
    for n in boards:
        x = torch.relu(torch.randn(n, 81, 128, generator=g)).cuda()
        r = torch.randn(n, 81, 128, generator=g).cuda()
        xa = board_amax(x)
        row = {"boards": n}
        for res in (None, r):
            tag = "res" if res is not None else "plain"
            set_conv_split(1)
            y0 = conv3x3_wino3h(x, u, su, b, res, x_amax=xa)
            row[f"persistent_{tag}_us"] = timeit(lambda: conv3x3_wino3h(x, u, su, b, res, x_amax=xa))
            set_conv_split(-1)
            row[f"product_{tag}_us"] = timeit(lambda: conv3x3_wino3h(x, u, su, b, res, x_amax=xa))
            y = torch.empty_like(x)
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            for split in (2, 4):
                for pf in (3, 6, 9, 12):
                    def run():
                        _lib.check(dl.uttt_diag_wino3s(p(x), p(u), su, p(b), p(res), p(y), p(xa), n, split, pf, st))
                    run()
                    torch.cuda.synchronize()
                    row[f"s{split}pf{pf}_{tag}_us"] = timeit(run)
                    if not torch.equal(y, y0):
                        row[f"s{split}pf{pf}_{tag}_bits_differ"] = True
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

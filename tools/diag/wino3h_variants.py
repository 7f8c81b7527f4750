#!/usr/bin/env python3
"""Time k_wino3h_conv pipeline variants (libuttt_diag.so uttt_diag_wino3h_variant) against the product
launch, plain and residual form, at the given board counts, interleaved A B A B to share the clock
state; each variant's output must equal the product's bit for bit.
usage: VARIANTS=1,6 python tools/diag/wino3h_variants.py 1344 2688 16384"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import torch  # noqa: E402
from uttt_amd import _lib  # noqa: E402
from uttt_amd.model import fold_bn, random_network  # noqa: E402
from uttt_amd.nnfast import board_amax, wino3h_weights, _p  # noqa: E402


def timeit(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    _lib.load()
    dlib = _lib.load_diag()
    f = dlib.uttt_diag_wino3h_variant
    f.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_float] + [ctypes.c_void_p] * 4 + [ctypes.c_int32] * 2 + \
        [ctypes.c_void_p]
    f.restype = ctypes.c_int
    net = random_network(0)
    w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
    uh, su = wino3h_weights(w)
    uh, b = uh.cuda(), b.cuda()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    variants = [int(v) for v in os.environ.get("VARIANTS", "1,6").split(",") if v]
    rounds = int(os.environ.get("ROUNDS", "3"))
    for n in [int(a) for a in (sys.argv[1:] or ["1344", "2688", "16384"])]:
        g = torch.Generator(device="cuda").manual_seed(n)
        x = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
        r = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
        ba = board_amax(x)
        outs = {}
        times = {}
        for res in (None, r):
            for v in [0] + variants:
                y = torch.empty_like(x)
                rc = f(_p(x), _p(uh), ctypes.c_float(su), _p(b), _p(res) if res is not None else None, _p(y), _p(ba), n, v, st)
                assert rc == 0, rc
                torch.cuda.synchronize()
                outs[(v, res is not None)] = y
        same = {f"{v}{'r' if rs else ''}": bool(torch.equal(outs[(v, rs)], outs[(0, rs)]))
                for v in variants for rs in (False, True)}
        for _ in range(rounds):
            for res in (None, r):
                for v in [0] + variants:
                    y = outs[(v, res is not None)]
                    t = timeit(lambda: f(_p(x), _p(uh), ctypes.c_float(su), _p(b), _p(res) if res is not None else None,
                                         _p(y), _p(ba), n, v, st))
                    times.setdefault(f"{v}{'r' if res is not None else ''}", []).append(round(t, 1))
        print(json.dumps({"boards": n, "us": times, "bits_equal_product": same}), flush=True)


if __name__ == "__main__":
    main()

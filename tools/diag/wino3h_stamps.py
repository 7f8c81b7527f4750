#!/usr/bin/env python3
"""Phase stamps of k_wino3h_conv (MODE 4): median core cycles per chunk phase over
workgroups 0..63, for wave 0 (SIMD 0, first half) and wave 4 (its SIMD partner)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]
from uttt_amd import _lib  # noqa: E402
from uttt_amd.model import fold_bn, random_network  # noqa: E402
from uttt_amd.nnfast import amax, wino3h_weights, _p  # noqa: E402

lib = _lib.load()
dlib = _lib.load_diag()
dlib.uttt_diag_wino3h_ablation.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_float] + [ctypes.c_void_p] * 3 + \
    [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
net = random_network(0)
w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
uh, su = wino3h_weights(w)
uh, b = uh.cuda(), b.cuda()
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
MODES = [int(v) for v in os.environ.get("MODES", "4").split(",")]
for n, mode in [(int(a), m) for a in (sys.argv[1:] or ["1344"]) for m in MODES]:
    x = torch.relu(torch.randn(n, 81, 128, device="cuda"))
    y = torch.empty_like(x)
    xa = amax(x)
    for _ in range(5):
        dlib.uttt_diag_wino3h_ablation(_p(x), _p(uh), ctypes.c_float(su), _p(b), _p(y), _p(xa), n, mode, st)
    torch.cuda.synchronize()
    ph = np.zeros((64, 2, 8, 6), np.uint32)
    assert dlib.uttt_diag_wino3h_stamps(ph.ctypes.data_as(ctypes.c_void_p)) == 0
    med = np.median(ph.astype(np.float64), axis=0)
    print(f"boards {n} mode {mode}: phase cycles (median over 64 WGs), cumulative -> deltas")
    names = ["load_x", "transform", "barrier+store_x", "gemm", "epilogue", "barrier"]
    for wv in range(2):
        print(f"  wave {4 * wv}")
        for c in range(4, 8):
            cum = med[wv, c]
            d = np.diff(np.concatenate([[0.0], cum]))
            print("   chunk %d: " % c + "  ".join(f"{nm} {int(v):6d}" for nm, v in zip(names, d)) + f"  total {int(cum[-1])}")

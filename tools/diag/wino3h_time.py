#!/usr/bin/env python3
"""Time k_wino3h_conv (split-f16 MFMA) at bench-like and large batches, plus its ablations
(1 no transform, 2 no point GEMMs, 64 no fold, ...) and prefetch-distance variants.
Accuracy vs f64 printed alongside."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from uttt_amd import _lib  # noqa: E402
from uttt_amd.model import fold_bn, random_network  # noqa: E402
from uttt_amd.nnfast import amax, board_amax, conv3x3_wino3h, wino3h_weights, _p  # noqa: E402


def timeit(fn, reps=20):
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
    lib = _lib.load()
    dlib = _lib.load_diag()
    dlib.uttt_diag_wino3h_ablation.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_float] + [ctypes.c_void_p] * 3 + \
        [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    net = random_network(0)
    w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
    uh, su = wino3h_weights(w)
    uh, b, wc = uh.cuda(), b.cuda(), w.cuda()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = []
    for n in [int(a) for a in (sys.argv[1:] or ["2048", "4096", "16384"])]:
        x = torch.relu(torch.randn(n, 81, 128, device="cuda"))
        y = torch.empty_like(x)
        xa = amax(x)
        ba = board_amax(x)
        th = timeit(lambda: lib.uttt_nn_conv3x3_wino3h(_p(x), _p(uh), ctypes.c_float(su), _p(b), None, _p(y), _p(ba), 1,
                                                      None, None, 0, n, st))
        r = torch.randn_like(x)
        th_res = timeit(lambda: lib.uttt_nn_conv3x3_wino3h(_p(x), _p(uh), ctypes.c_float(su), _p(b), _p(r), _p(y),
                                                          _p(ba), 1, None, None, 0, n, st))
        abl = {m: timeit(lambda m=m: dlib.uttt_diag_wino3h_ablation(_p(x), _p(uh), ctypes.c_float(su), _p(b), _p(y),
                                                                    _p(xa), n, m, st)) for m in [int(v) for v in os.environ.get("MODES", "1,2,8,64,16,32,48,49,112,512").split(",")]}
        dlib.uttt_diag_wino3h_pf.argtypes = dlib.uttt_diag_wino3h_ablation.argtypes
        for pf in [int(v) for v in os.environ.get("PFS", "").split(",") if v]:
            abl["pf%d" % pf] = timeit(lambda pf=pf: dlib.uttt_diag_wino3h_pf(_p(x), _p(uh), ctypes.c_float(su), _p(b),
                                                                            _p(y), _p(xa), n, pf, st))
        xs = x[:min(n, 512)]
        ref = F.conv2d(xs.reshape(-1, 9, 9, 128).permute(0, 3, 1, 2).double(), wc.double(), b.double(), padding=1)
        ref = torch.relu(ref).permute(0, 2, 3, 1).reshape(-1, 81, 128)
        yh = conv3x3_wino3h(xs, uh, su, b)
        torch.cuda.synchronize()
        sc = ref.abs().max().item()
        u8 = uh.repeat(8)
        abl[256] = timeit(lambda: dlib.uttt_diag_wino3h_ablation(_p(x), _p(u8), ctypes.c_float(su), _p(b), _p(y),
                                                                _p(xa), n, 256, st))
        rec = {"boards": n, "wino3h_us": round(th, 1), "wino3h_res_us": round(th_res, 1), "ablation_us": {str(k): round(v, 1) for k, v in abl.items()},
               "direct_equiv_tflops": round(2 * 81 * 128 * 1152 * n / th / 1e6, 1),
               "err_rel_wino3h": (yh.double() - ref).abs().max().item() / sc}
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()

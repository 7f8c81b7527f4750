"""Runs k_wino3_conv (full, mode 0) 10x at n boards: a target for rocprofv3 --pmc passes."""
import ctypes, sys
import torch
sys.path[:0] = ['.', 'ultimate-tictactoe-alphazero_amd']
from uttt_amd import _lib
from uttt_amd.nnfast import wino3_weights, _p
from uttt_amd.model import fold_bn, random_network
lib = _lib.load()
lib.uttt_diag_wino3_ablation.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
net = random_network(0)
w, b = fold_bn(net.residual_blocks[0].conv1, net.residual_blocks[0].bn1)
u = wino3_weights(w).cuda(); b = b.cuda()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
x = torch.relu(torch.randn(n, 81, 128)).cuda(); y = torch.empty_like(x)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(10):
    lib.uttt_diag_wino3_ablation(_p(x), _p(u), _p(b), _p(y), n, mode, st)
torch.cuda.synchronize()
print("ok")
if mode & 4:
    mhz, us = ctypes.c_double(), ctypes.c_double()
    assert lib.uttt_diag_wino3_clock(ctypes.byref(mhz), ctypes.byref(us)) == 0
    print(f"median shader clock {mhz.value:.0f} MHz, median workgroup {us.value:.2f} us")
    import numpy as np
    ph = np.zeros((64, 2, 40), np.uint32)
    assert lib.uttt_diag_wino3_phases(ph.ctypes.data_as(ctypes.c_void_p)) == 0
    med = np.median(ph[8:56].astype(np.float64), axis=0)   # skip first/last launches' edge WGs
    for w, nm in ((0, "wave0"), (1, "wave4")):
        print(nm, "prologue", int(med[w, 0]) if w == 0 else "-")
        for c in range(8):
            t, g, ba, bb = med[w, 1 + 4 * c:5 + 4 * c]
            print(f"  chunk {c}: transform {int(t):6d}  gemm {int(g):6d}  barrierA {int(ba):6d}  store+barrierB {int(bb):6d}")

"""Timing ablations of the Winograd conv kernels at n boards (one process, interleaved, median of 20):
F(2x2,3x3) k_wino_conv, F(3x3,3x3) k_wino3_conv, MIOpen direct conv for reference."""
import ctypes, sys
import torch
sys.path[:0] = ['.', 'ultimate-tictactoe-alphazero_amd']
from uttt_amd import _lib
from uttt_amd.nnfast import wino_weights, wino3_weights, _p
from uttt_amd.model import fold_bn, random_network
import torch.nn.functional as F
lib = _lib.load()
for f in ("uttt_diag_wino_ablation", "uttt_diag_wino3_ablation"):
    getattr(lib, f).argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
net = random_network(0)
w, b = fold_bn(net.residual_blocks[0].conv1, net.residual_blocks[0].bn1)
u2 = wino_weights(w).cuda(); u3 = wino3_weights(w).cuda(); b = b.cuda()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
x = torch.relu(torch.randn(n, 81, 128)).cuda(); y = torch.empty_like(x)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
names = {0: "full", 1: "no-transform", 2: "no-gemm", 3: "no-fold"}
names3 = {**names, 65: "no-transform no-fold", 512: "unpinned MFMAs"}
wc = w.cuda().contiguous(memory_format=torch.channels_last)
xn = x.reshape(n, 9, 9, 128).permute(0, 3, 1, 2)
cases = {}
for m, nm in names.items():
    cases[f"F2 {nm}"] = lambda m=m: lib.uttt_diag_wino_ablation(_p(x), _p(u2), _p(b), _p(y), n, m, st)
for m, nm in names3.items():
    cases[f"F3 {nm}"] = lambda m=m: lib.uttt_diag_wino3_ablation(_p(x), _p(u3), _p(b), _p(y), n, m, st)
cases["miopen"] = lambda: F.conv2d(xn, wc, None, padding=1)
times = {k: [] for k in cases}
for it in range(22):
    for k, fn in cases.items():
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); e.record()
        torch.cuda.synchronize()
        if it >= 2: times[k].append(a.elapsed_time(e))
flop_direct = n * 81 * 128 * 1152 * 2
exe = {"F2": n * 25 * 16 * 128 * 128 * 2, "F3": n * 9 * 25 * 128 * 128 * 2, "mi": flop_direct}
print(f"n = {n} boards")
for k, ts in times.items():
    ts.sort(); med = ts[len(ts) // 2]
    print(f"{k:>16}: {med*1e3:8.1f} us   direct-equiv {flop_direct/med/1e9:7.1f} TF/s   "
          f"mfma-executed {exe[k[:2]]/med/1e9:7.1f} TF/s", flush=True)

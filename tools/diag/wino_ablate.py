"""Timing ablations of k_wino_conv at n=4096 boards (one process, interleaved, median of 20)."""
import ctypes, sys
import torch
sys.path[:0] = ['.', 'ultimate-tictactoe-alphazero_amd']
from uttt_amd import _lib
from uttt_amd.nnfast import wino_weights, _p
from uttt_amd.model import fold_bn, random_network
import torch.nn.functional as F
lib = _lib.load()
lib.uttt_diag_wino_ablation.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
net = random_network(0)
w, b = fold_bn(net.residual_blocks[0].conv1, net.residual_blocks[0].bn1)
u = wino_weights(w).cuda(); b = b.cuda()
n = 4096
x = torch.relu(torch.randn(n, 81, 128)).cuda(); y = torch.empty_like(x)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
names = {0: "full", 1: "no-transform", 2: "no-gemm", 3: "no-fold"}
times = {m: [] for m in names}
wc = w.cuda().contiguous(memory_format=torch.channels_last)
xn = x.reshape(n, 9, 9, 128).permute(0, 3, 1, 2)
times["miopen"] = []
for it in range(22):
    for m in names:
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); lib.uttt_diag_wino_ablation(_p(x), _p(u), _p(b), _p(y), n, m, st); e.record()
        torch.cuda.synchronize()
        if it >= 2: times[m].append(a.elapsed_time(e))
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); F.conv2d(xn, wc, None, padding=1); e.record(); torch.cuda.synchronize()
    if it >= 2: times["miopen"].append(a.elapsed_time(e))
flop_direct = n * 81 * 128 * 1152 * 2
flop_mfma = n * 25 * 16 * 128 * 128 * 2
for m, ts in times.items():
    ts.sort(); med = ts[len(ts) // 2]
    print(f"{names.get(m, m):>13}: {med*1e3:8.1f} us   direct-equiv {flop_direct/med/1e9:7.1f} TF/s   mfma-executed {flop_mfma/med/1e9:7.1f} TF/s", flush=True)

"""Do two small k_wino3_conv launches on two streams run concurrently? (events per stream)"""
import ctypes, sys, time
import torch
sys.path[:0] = ['.', 'ultimate-tictactoe-alphazero_amd']
from uttt_amd import _lib
from uttt_amd.nnfast import wino3_weights, _p
from uttt_amd.model import fold_bn, random_network
lib = _lib.load()
net = random_network(0)
w, b = fold_bn(net.residual_blocks[0].conv1, net.residual_blocks[0].bn1)
u = wino3_weights(w).cuda(); b = b.cuda()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
reps = 50
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
xs = [torch.relu(torch.randn(n, 81, 128)).cuda() for _ in range(2)]
ys = [torch.empty_like(xs[0]) for _ in range(2)]
def run(streams):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                lib.uttt_nn_conv3x3_wino3(_p(xs[i]), _p(u), _p(b), None, _p(ys[i]), n, ctypes.c_void_p(st.cuda_stream))
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6
run([s1, s2])
one = run([s1])
same = run([s1, s1])
two = run([s1, s2])
print(f"n={n}: one conv {one:.1f} us, two on one stream {same:.1f} us, two on two streams {two:.1f} us")

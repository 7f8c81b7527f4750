#!/usr/bin/env python3
"""k_heads before / after a restructuring, same inputs: the policy (softmax and logits) and value
bits must be equal. The previous kernel is built from the previous commit's csrc/nn_kernels.hip
into ultimate-tictactoe-alphazero_amd/build/prev/libuttt_heads_prev.so (heads)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")
sys.path[:0] = [PKG]

import torch  # noqa: E402
from uttt_amd import _lib  # noqa: E402
from uttt_amd.model import calibrated_network, random_network  # noqa: E402
from uttt_amd.nnfast import _p, pack_heads  # noqa: E402


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
    new = _lib.load()
    prev = ctypes.CDLL(os.path.join(PKG, "build", "prev", "libuttt_heads_prev.so"))
    for lib in (new, prev):
        lib.uttt_nn_heads.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int32] + [ctypes.c_void_p] * 2 + \
            [ctypes.c_int32, ctypes.c_void_p]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out, us = {}, {}
    nets = {"seed0": random_network(0),
            "calibrated": calibrated_network(os.path.join(REPO, "tests", "golden", "netcal.npz"))}
    for name, net in nets.items():
        hw = pack_heads(net, "cuda")
        for n in (1, 7, 8, 9, 1381, 2048):
            g = torch.Generator(device="cuda").manual_seed(n)
            act = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
            for sm in (1, 0):
                res = []
                for tag, lib in (("new", new), ("prev", prev)):
                    p = torch.zeros(n, 81, device="cuda")
                    v = torch.zeros(n, device="cuda")
                    assert lib.uttt_nn_heads(_p(act), _p(hw), n, _p(p), _p(v), sm, st) == 0
                    torch.cuda.synchronize()
                    res.append((p, v))
                    if name == "seed0" and sm == 1 and n >= 1381:
                        us[f"{tag}/n{n}"] = round(timeit(lambda: lib.uttt_nn_heads(_p(act), _p(hw), n, _p(p), _p(v),
                                                                                    sm, st)), 1)
                out[f"{name}/n{n}/softmax{sm}"] = bool(torch.equal(res[0][0], res[1][0]) and
                                                        torch.equal(res[0][1], res[1][1]))
    print(json.dumps({"bits_equal": out, "all": all(out.values()), "us": us}), flush=True)
    assert all(out.values())


if __name__ == "__main__":
    main()

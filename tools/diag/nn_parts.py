#!/usr/bin/env python3
"""Time the evaluator's non-conv kernels (stem from packed states, heads) at N positions with
HIP events; prints us per launch. usage: nn_parts.py 1344"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd"), os.path.join(REPO, "tools", "diag")]
import uttt_amd  # noqa: E402
from uttt_amd.model import random_network  # noqa: E402
from uttt_amd.nnfast import FusedNetworkEvaluator, _p  # noqa: E402


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


n = int(sys.argv[1]) if len(sys.argv) > 1 else 1344
fe = FusedNetworkEvaluator(random_network(0, "cuda"), None, max_batch=n)
states = uttt_amd.initial_states(n)
st = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
st.copy_(torch.from_numpy(states.view("<i4").reshape(n, 8)))
lib = fe.lib
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
t_stem = timeit(lambda: lib.uttt_nn_stem_states(_p(st), n, _p(fe.stem_w), _p(fe.stem_b), _p(fe.buf[0]), s))
t_heads = timeit(lambda: lib.uttt_nn_heads(_p(fe.buf[0]), _p(fe.heads), n, _p(fe.policy), _p(fe.value), 1, s))
print(json.dumps({"boards": n, "stem_us": round(t_stem, 1), "heads_us": round(t_heads, 1)}))

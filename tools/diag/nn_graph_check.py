#!/usr/bin/env python3
"""The fused evaluator's forward (stem + 32 tower convs + heads, device-count form) as 34 launches against
the same launches captured once into a HIP graph (torch.cuda.CUDAGraph) and replayed: us per forward at a
few board counts, and the outputs bit-equal. One JSON line."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import uttt_amd  # noqa: E402
from uttt_amd.model import random_network  # noqa: E402
from uttt_amd.nnfast import FusedNetworkEvaluator, _p  # noqa: E402


def main():
    out = {}
    for n in (8, 1370, 4096):
        fe = FusedNetworkEvaluator(random_network(0, "cuda"), None, max_batch=max(n, 8))
        states = uttt_amd.initial_states(n)
        st = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
        st.copy_(torch.from_numpy(np.ascontiguousarray(states).view(np.int32).reshape(n, 8)))
        n_dev = torch.tensor([n], dtype=torch.int32, device="cuda")
        lib = fe.lib
        s = torch.cuda.Stream()
        torch.cuda.synchronize()

        def forward():
            stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            lib.uttt_nn_stem_states(_p(st), n, _p(fe.stem_w), _p(fe.stem_b), _p(fe.buf[0]), stream)
            fe._tower_heads(n, True, n_dev=ctypes.c_void_p(n_dev.data_ptr()))

        with torch.cuda.stream(s):
            for _ in range(3):
                forward()
            torch.cuda.synchronize()
            ref = (fe.policy[:n].clone(), fe.value[:n].clone())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                forward()
            e1.record()
            torch.cuda.synchronize()
            t_plain = e0.elapsed_time(e1) * 1e3 / 50
            fe._plan = None  # the capture builds its plan on the capture stream
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                forward()
            g.replay()
            torch.cuda.synchronize()
            same = bool(torch.equal(ref[0], fe.policy[:n]) and torch.equal(ref[1], fe.value[:n]))
            e0.record()
            for _ in range(50):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            t_graph = e0.elapsed_time(e1) * 1e3 / 50
        out[n] = {"launches_us": round(t_plain, 1), "graph_us": round(t_graph, 1), "bits_equal": same}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

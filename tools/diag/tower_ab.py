#!/usr/bin/env python3
"""The residual tower as ONE dataflow launch (uttt_nn_tower_wino3h_dev, round 6) against the 32
per-conv launches (uttt_nn_conv3x3_wino3h), timed interleaved A B A B on one box, with the output bits
compared. Positions: random legal play from the initial state (seeded), the calibrated network.

  python tools/diag/tower_ab.py [JSON_OUT] [N,N,...] [ROUNDS] [REPS]

Per N and round: REPS towers of each form back to back between HIP events on the current stream
(stem and heads excluded: both forms share them). Prints one JSON document."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]
import uttt_amd  # noqa: E402
from uttt_amd._lib import UtttState  # noqa: E402
from uttt_amd.model import calibrated_network  # noqa: E402
from uttt_amd.nnfast import FusedNetworkEvaluator  # noqa: E402

out_path = sys.argv[1] if len(sys.argv) > 1 else None
sizes = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1370,2740,4096,16384").split(",")]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
EXEC_FLOP = 22.12e6  # executed f16 MFMA flops per board per conv (bench.py CONV_EXEC_FLOP)
PEAK = 2500.0


def positions(n, seed=0):
    rng = np.random.RandomState(seed)
    states = uttt_amd.initial_states(n)
    lib = uttt_amd._lib.load()
    leg = (ctypes.c_int32 * 81)()
    for i in range(n):
        s = UtttState.from_buffer(states[i:i + 1])
        for _ in range(rng.randint(0, 40)):
            nl = lib.uttt_state_legal_actions(ctypes.byref(s), leg)
            if nl == 0:
                break
            t = UtttState()
            lib.uttt_state_next(ctypes.byref(s), leg[rng.randint(nl)], ctypes.byref(t))
            ctypes.memmove(ctypes.addressof(s), ctypes.addressof(t), 32)
    return states


net = calibrated_network(os.path.join(REPO, "tests", "golden", "netcal.npz"), "cuda")
res = {"method": "interleaved A (per-conv launches) / B (dataflow tower) on one box; HIP events around REPS towers",
       "rounds": rounds, "reps": reps, "points": []}
for n in sizes:
    st = positions(n, seed=n)
    fe = {k: FusedNetworkEvaluator(net, None, max_batch=n, tower=k) for k in ("layers", "dataflow")}
    outs = {}
    for k, f in fe.items():
        p, v = f.forward_states(st)  # stem + tower + heads; buf[0] = the tower's output
        outs[k] = (p.clone(), v.clone(), f.buf[0][:n].clone())
    same = all(torch.equal(a, b) for a, b in zip(outs["layers"], outs["dataflow"]))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    times = {"layers": [], "dataflow": []}
    for r in range(rounds):
        for k in ("layers", "dataflow"):
            f = fe[k]
            f.forward_states(st)  # warm (the stem output is left in buf[0])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # the tower alone, REPS times on the same stem output (buf[0] is the tower's input and output:
            # re-run the stem between towers so every tower starts from the same activations)
            tot = 0.0
            for i in range(reps):
                check = uttt_amd._lib.check
                check(f.lib.uttt_nn_stem_states(ctypes.c_void_p(f.states.data_ptr()), n, ctypes.c_void_p(f.stem_w.data_ptr()),
                                                ctypes.c_void_p(f.stem_b.data_ptr()), ctypes.c_void_p(f.buf[0].data_ptr()),
                                                stream))
                e0.record()
                if k == "dataflow":
                    f._tower_dataflow(stream, None, n)
                else:
                    f.tower = "layers"
                    f.tower_events = []
                    f._tower_heads(n, True)  # per-conv launches + heads; the heads are timed apart below
                    f.tower_events = None
                e1.record()
                torch.cuda.synchronize()
                tot += e0.elapsed_time(e1)
            times[k].append(tot * 1e3 / reps)
    # the heads alone (the layers form's events include them)
    f = fe["layers"]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        uttt_amd._lib.check(f.lib.uttt_nn_heads(ctypes.c_void_p(f.buf[0].data_ptr()), ctypes.c_void_p(f.heads.data_ptr()), n,
                                                ctypes.c_void_p(f.policy.data_ptr()), ctypes.c_void_p(f.value.data_ptr()), 1,
                                                stream))
    e1.record()
    torch.cuda.synchronize()
    heads_us = e0.elapsed_time(e1) * 1e3 / reps
    lay = [t - heads_us for t in times["layers"]]
    dfl = times["dataflow"]
    pt = {"boards": n, "bits_equal": bool(same), "heads_us": round(heads_us, 1),
          "layers_tower_us": [round(t, 1) for t in lay], "dataflow_tower_us": [round(t, 1) for t in dfl],
          "layers_frac": round(EXEC_FLOP * 32 * n / (min(lay) * 1e-6) / 1e12 / PEAK, 4),
          "dataflow_frac": round(EXEC_FLOP * 32 * n / (min(dfl) * 1e-6) / 1e12 / PEAK, 4),
          "speedup_median": round(float(np.median(lay)) / float(np.median(dfl)), 4)}
    res["points"].append(pt)
    print(json.dumps(pt), flush=True)
    del fe
    torch.cuda.empty_cache()
if out_path:
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)

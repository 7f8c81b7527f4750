#!/usr/bin/env python3
"""Target for rocprofv3 --pmc passes on the leaf evaluator: the fused DualNetwork (stem, 32
split-f16 Winograd convs, heads) on N positions (default 1344, about one lane's batch at the
bench config), REPS forwards. Positions: random legal play from the initial state (seeded)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]
import uttt_amd  # noqa: E402
from uttt_amd.model import random_network  # noqa: E402
from uttt_amd.nnfast import FusedNetworkEvaluator  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1344
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
import ctypes  # noqa: E402
from uttt_amd._lib import UtttState  # noqa: E402

rng = np.random.RandomState(0)
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
fe = FusedNetworkEvaluator(random_network(0, "cuda"), None, max_batch=n)
for _ in range(reps):
    fe.forward_states(states)
torch.cuda.synchronize()
print(f"nn_forward_only: {reps} forwards x {n} positions")

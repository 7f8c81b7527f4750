"""TEST INFRASTRUCTURE ONLY — numpy twin of the deterministic hash evaluator.

Same spec as or_hash_eval (oracle/uttt_oracle.c) and the device evaluator
(csrc/uttt_hash.h): bits of the NCHW (3,9,9) input -> 4 u64 words -> splitmix
finaliser chain -> 81 priors (24-bit / 2^24, with the zero / subnormal / sparse
modes) and a value in {-1, -0.999, ..., 1}.

``HashModel`` is a torch.nn.Module with the DualNetwork call signature
(``model(x) -> (policies (N,81) f32, values (N,1) f32)``) so the reference's own
Python driver (pv_mcts_cpp.inference_func / self_play_cpp.play) can be run on it
to produce golden self-play fixtures.
"""
import numpy as np

M64 = (1 << 64) - 1
GOLD = 0x9E3779B97F4A7C15


def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def hash_eval_np(x, salt=0):
    """salt != 0: a different deterministic player (h = mix64(h ^ salt))."""
    x = np.asarray(x, dtype=np.float32).reshape(243)
    w = [0, 0, 0, 0]
    for j in np.nonzero(x != 0.0)[0].tolist():
        w[j >> 6] |= 1 << (j & 63)
    h = GOLD
    for i in range(4):
        h = mix64(h ^ w[i])
    if salt:
        h = mix64(h ^ salt)
    mode = (h >> 8) & 15
    pol = np.zeros(81, np.float32)
    scale = np.float32(1.0 / 16777216.0)
    tiny = np.float32(2.0 ** -140)
    for a in range(81):
        r = mix64(h + (a + 1) * GOLD)
        p = np.float32(r >> 40) * scale
        if mode == 0:
            p = np.float32(0.0)
        elif mode == 1:
            p = np.float32(p * tiny)
        elif mode == 2 and (a & 3):
            p = np.float32(0.0)
        pol[a] = p
    rv = mix64(h ^ 0xD6E8FEB86659FD93)
    val = np.float32(int(rv % 2001) - 1000) / np.float32(1000.0)
    return pol, np.float32(val)


def make_hash_model(salt=0):
    import torch

    class HashModel(torch.nn.Module):
        """DualNetwork-shaped deterministic evaluator (no parameters)."""

        def forward(self, x):
            xs = x.detach().cpu().numpy().reshape(x.shape[0], 243)
            pols = np.zeros((xs.shape[0], 81), np.float32)
            vals = np.zeros((xs.shape[0], 1), np.float32)
            for i in range(xs.shape[0]):
                pols[i], vals[i, 0] = hash_eval_np(xs[i], salt)
            return torch.from_numpy(pols).to(x.device), torch.from_numpy(vals).to(x.device)

    return HashModel()

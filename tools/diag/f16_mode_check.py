#!/usr/bin/env python3
"""The tower conv's f16 mode (uttt_nn_conv3x3_wino3h_f16: M = Vhi Uhi only) against the product split-f16
conv: error vs an f64 direct conv per board (max |err| / the board's max |y|), the whole network's value and
policy vs the fp32 DualNetwork on search leaves, and the two convs' launch times interleaved (plain and
residual, 1,370 and 16,384 boards). Prints one JSON line."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from uttt_amd import _lib  # noqa: E402
from uttt_amd.model import fold_bn, random_network, calibrated_network  # noqa: E402
from uttt_amd.nnfast import FusedNetworkEvaluator, board_amax, conv3x3_wino3h, wino3h_weights, _p  # noqa: E402


def conv_errors():
    net = random_network(3)
    g = torch.Generator().manual_seed(2)
    out = []
    for blk_i, n, scale in ((5, 7, 1.0), (15, 64, 1e3), (9, 1000, 1.0), (2, 257, 1e-3)):
        w, b = fold_bn(net.residual_blocks[blk_i].conv1, net.residual_blocks[blk_i].bn1)
        u, su = wino3h_weights(w)
        u, w, b = u.cuda(), w.cuda(), b.cuda()
        x = (torch.relu(torch.randn(n, 81, 128, generator=g)) * scale).cuda()
        r = (torch.randn(n, 81, 128, generator=g) * scale).cuda()
        ref = F.conv2d(x.reshape(n, 9, 9, 128).permute(0, 3, 1, 2).double(), w.double(), b.double(),
                       padding=1).permute(0, 2, 3, 1).reshape(n, 81, 128)
        for res in (None, r):
            want = torch.relu(ref + (res.double() if res is not None else 0)).float()
            bscale = want.abs().reshape(n, -1).amax(dim=1).clamp_min(1e-30)
            rec = {"block": blk_i, "boards": n, "scale": scale, "residual": res is not None}
            for prec in ("f32", "f16"):
                y = conv3x3_wino3h(x, u, su, b, res, precision=prec)
                rec[prec] = float(((y - want).abs().reshape(n, -1).amax(dim=1) / bscale).max())
            # batch independence of the f16 mode: the first 5 boards alone give the same bits
            y_all = conv3x3_wino3h(x, u, su, b, res, precision="f16")
            y_5 = conv3x3_wino3h(x[:5].contiguous(), u, su, b, res[:5].contiguous() if res is not None else None,
                                 precision="f16")
            rec["f16_batch_independent"] = bool(torch.equal(y_all[:5], y_5))
            out.append(rec)
    return out


def network_errors():
    import uttt_cpp
    from uttt_amd._lib import STATE_DTYPE
    from uttt_amd.model import policy_logits
    rng = np.random.default_rng(5)
    states = []
    while len(states) < 400:  # positions along random games (the drop-in module's rules)
        s = uttt_cpp.State()
        while not s.is_done() and len(states) < 400:
            if rng.random() < 0.3:
                states.append(s)
            s = s.next(int(rng.choice(s.legal_actions())))
    packed = np.frombuffer(b"".join(s.packed for s in states), dtype=STATE_DTYPE)
    x = torch.tensor(np.array([s.to_input_tensor() for s in states], np.float32)).reshape(-1, 9, 9, 3).permute(0, 3, 1, 2)
    netcal = os.path.join(REPO, "tests", "golden", "netcal.npz")
    res = {}
    for name, make in (("seed0", lambda d: random_network(0, d)), ("calibrated", lambda d: calibrated_network(netcal, d))):
        z_cpu, v_cpu = policy_logits(make("cpu"), x.contiguous())
        p_cpu = torch.softmax(z_cpu, dim=1)
        for prec in ("f32", "f16"):
            ev = FusedNetworkEvaluator(make("cuda"), max_batch=len(states), precision=prec)
            p, v = ev.forward_states(packed)
            res[f"{name}_{prec}"] = {"value_max_abs": float((v.cpu() - v_cpu.reshape(-1)).abs().max()),
                                     "policy_max_abs": float((p.cpu() - p_cpu).abs().max())}
    return res


def search_agreement():
    """The same 50-simulation searches (B = 8) from 400 positions with the calibrated net through the f32-level
    evaluator and through the f16 mode: how often the most-visited root action agrees, and the mean total
    variation distance between the two visit distributions (a network 1e-2 off moves the searches this much)."""
    import uttt_cpp
    from uttt_amd import BatchedSearch
    from uttt_amd._lib import STATE_DTYPE
    rng = np.random.default_rng(9)
    states = []
    while len(states) < 400:
        s = uttt_cpp.State()
        while not s.is_done() and len(states) < 400:
            if rng.random() < 0.3:
                states.append(s)
            s = s.next(int(rng.choice(s.legal_actions())))
    roots = np.frombuffer(b"".join(s.packed for s in states), dtype=STATE_DTYPE)
    net = calibrated_network(os.path.join(REPO, "tests", "golden", "netcal.npz"), "cuda")
    out = {}
    for prec in ("f32", "f16"):
        bs = BatchedSearch(len(states), 50)
        bs.run(roots, FusedNetworkEvaluator(net, bs.engine, precision=prec), 50, 8)
        out[prec] = bs.visits()
    (v32, L), (v16, _) = out["f32"], out["f16"]
    agree = [int(np.argmax(v32[i, :L[i]]) == np.argmax(v16[i, :L[i]])) for i in range(len(states))]
    tv = [0.5 * float(np.abs(v32[i, :L[i]] / 50.0 - v16[i, :L[i]] / 50.0).sum()) for i in range(len(states))]
    return {"positions": len(states), "top_action_agreement": float(np.mean(agree)), "mean_visit_tv": float(np.mean(tv)),
            "identical_visits": float(np.mean([np.array_equal(v32[i], v16[i]) for i in range(len(states))]))}


def timing():
    lib = _lib.load()
    net = random_network(0)
    w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
    uh, su = wino3h_weights(w)
    uh, b = uh.cuda(), b.cuda()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for n in (1370, 16384):
        g = torch.Generator(device="cuda").manual_seed(n)
        x = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
        r = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
        ba = board_amax(x)
        y = torch.empty_like(x)
        fns = {"f32": lib.uttt_nn_conv3x3_wino3h, "f16": lib.uttt_nn_conv3x3_wino3h_f16}
        times = {}
        for _ in range(5):
            for prec, fn in fns.items():
                for res in (None, r):
                    call = lambda: fn(_p(x), _p(uh), ctypes.c_float(su), _p(b), _p(res) if res is not None else None,
                                      _p(y), _p(ba), 1, None, None, 0, n, st)
                    call()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(20):
                        call()
                    e1.record()
                    torch.cuda.synchronize()
                    times.setdefault(prec + ("_res" if res is not None else ""), []).append(
                        round(e0.elapsed_time(e1) * 1e3 / 20, 1))
        out[n] = {k: {"median_us": float(np.median(v)), "us": v} for k, v in times.items()}
    return out


if __name__ == "__main__":
    print(json.dumps({"conv": conv_errors(), "network": network_errors(), "search": search_agreement(),
                      "timing_us": timing()}), flush=True)

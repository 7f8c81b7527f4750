"""CPU tests of the product's host side: the C-ABI library loads and exports
every function include/uttt_engine.h declares; the `uttt_cpp` State (bitboard
rules shared with the kernels) reproduces the reference's rules, transitions,
tensors and to_string on the golden fixtures; argument validation."""
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, REPO, golden


def _declared_functions():
    src = ""
    for h in ("uttt_engine.h", "uttt_nn.h"):
        with open(os.path.join(REPO, "include", h)) as f:
            src += f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\*?\s*(uttt_\w+)\s*\(", src, flags=re.M)))


def test_abi_exports_every_declared_symbol(engine_lib):
    names = _declared_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(engine_lib, n), n
    assert engine_lib.uttt_version().decode().startswith("uttt-mi355x")


def _st(m, d, i, prefix=""):
    return m.State(d[prefix + "pieces"][i].reshape(9, 9).tolist(), d[prefix + "enemy"][i].reshape(9, 9).tolist(),
                   d[prefix + "main_p"][i].tolist(), d[prefix + "main_e"][i].tolist(), int(d[prefix + "active"][i]))


def test_state_rules_match_reference(uttt_cpp_mod):
    m = uttt_cpp_mod
    d = golden("rules.npz")
    n = len(d["n_legal"])
    for i in range(n):
        s = _st(m, d, i)
        assert s.legal_actions() == np.nonzero(d["legal"][i])[0].tolist()
        fl = int(s.is_lose()) | int(s.is_draw()) << 1 | int(s.is_done()) << 2 | int(s.is_first_player()) << 3
        assert fl == d["flags"][i]
        assert np.array_equal(np.asarray(s.to_input_tensor(), np.float32), d["tensor"][i].astype(np.float32))
        assert s.pieces == d["pieces"][i].reshape(9, 9).tolist()
        assert s.main_board_enemy_pieces == d["main_e"][i].tolist()
        a = int(d["action"][i])
        if a >= 0 and i + 1 < n and d["game"][i + 1] == d["game"][i]:
            nx = s.next(a)
            assert nx.pieces == d["pieces"][i + 1].reshape(9, 9).tolist()
            assert nx.enemy_pieces == d["enemy"][i + 1].reshape(9, 9).tolist()
            assert nx.main_board_pieces == d["main_p"][i + 1].tolist()
            assert nx.main_board_enemy_pieces == d["main_e"][i + 1].tolist()
            assert nx.active_board == d["active"][i + 1]


def test_unvalidated_next_matches_reference(uttt_cpp_mod):
    m = uttt_cpp_mod
    d = golden("rules.npz")
    for i in range(len(d["odd_action"])):
        nx = _st(m, d, i, "odd_").next(int(d["odd_action"][i]))
        assert nx.pieces == d["odd_n_pieces"][i].reshape(9, 9).tolist()
        assert nx.enemy_pieces == d["odd_n_enemy"][i].reshape(9, 9).tolist()
        assert nx.main_board_pieces == d["odd_n_main_p"][i].tolist()
        assert nx.main_board_enemy_pieces == d["odd_n_main_e"][i].tolist()
        assert nx.active_board == d["odd_n_active"][i]


def test_to_string_matches_reference(uttt_cpp_mod):
    m = uttt_cpp_mod
    with open(os.path.join(GOLDEN, "to_string.json")) as f:
        items = json.load(f)
    for it in items:
        p, e, mp, me, a = it["state"]
        s = m.State(np.reshape(p, (9, 9)).tolist(), np.reshape(e, (9, 9)).tolist(), mp, me, a)
        assert s.to_string() == it["text"]
        assert str(s) == it["text"]


def test_state_validation_and_packing(uttt_cpp_mod):
    m = uttt_cpp_mod
    z = [[0] * 9 for _ in range(9)]
    with pytest.raises(ValueError):
        m.State([[2] * 9] + z[1:], z, [0] * 9, [0] * 9, -1)
    with pytest.raises(ValueError):
        m.State(z, z, [0] * 9, [0] * 9, 9)
    with pytest.raises(TypeError):
        m.State(z[:8], z, [0] * 9, [0] * 9, -1)
    with pytest.raises(ValueError):
        m.State().next(81)
    s = m.State().next(40)
    t = m.State.from_packed(s.packed)
    assert t.pieces == s.pieces and t.active_board == 4 and len(s.packed) == 32


def test_boltzman_matches_reference_values(uttt_cpp_mod, oracle_lib):
    rng = np.random.RandomState(5)
    for tau in (1.0, 0.5, 2.0, 0.25):
        xs = rng.randint(0, 60, size=rng.randint(1, 82)).astype(np.float32)
        a = np.asarray(uttt_cpp_mod.boltzman(xs.tolist(), tau), np.float32)
        b = oracle_lib.boltzman(xs, tau)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_engine_requires_gpu_loudly():
    """No silent CPU path: without a GPU the engine refuses to start."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from uttt_amd import Engine
    from uttt_amd._lib import EngineError
    with pytest.raises(EngineError):
        Engine(4, 50)


def test_engine_limits_are_checked_before_the_device(engine_lib):
    """max_sims is bounded by the 16-byte node record (visits, child-block counts <= 4095): larger
    requests are refused with UTTT_ERR_ARG and a message, before any device call."""
    import ctypes
    h = ctypes.c_void_p()
    assert engine_lib.uttt_engine_create(-1, 4, 4096, ctypes.byref(h)) == -1
    assert b"4095" in engine_lib.uttt_last_error()
    assert engine_lib.uttt_engine_create(-1, 0, 50, ctypes.byref(h)) == -1


def test_dropin_refuses_evaluate_count_above_the_node_record(uttt_cpp_mod):
    """uttt_cpp.pv_mcts_scores with evaluate_count > UTTT_MAX_SIMS (4095) raises ValueError naming
    the limit, before the model or the device is touched (the reference has no such bound;
    INTEGRATION.md §2 'Limit')."""
    called = []

    def model(states):
        called.append(len(states))
        return [(np.zeros(81, np.float32), 0.0) for _ in states]

    with pytest.raises(ValueError, match="4095"):
        uttt_cpp_mod.pv_mcts_scores(model=model, state=uttt_cpp_mod.State(), temperature=1.0,
                                    evaluate_count=4096, batch_size=8)
    assert not called


def test_calibrated_network_reproduces_reference_fixture():
    """tests/golden/netcal.npz pins the non-saturated network the GPU parity tests use: the
    seed-0 DualNetwork + the fixture's BatchNorm statistics (uttt_amd.model.calibrated_network)
    has the reference's parameters (per-tensor sums) and reproduces the reference's CPU fp32
    outputs; and the net is genuinely unsaturated."""
    import torch
    from uttt_amd.model import calibrated_network
    d = golden("netcal.npz")
    net = calibrated_network(os.path.join(GOLDEN, "netcal.npz"))
    sd = net.state_dict()
    sums = np.asarray([t.double().sum().item() for t in sd.values()])
    floats = np.asarray([t.is_floating_point() for t in sd.values()])  # not num_batches_tracked
    assert np.allclose(sums[floats], d["param_sums"][floats], rtol=1e-9, atol=1e-9)
    with torch.no_grad():
        p, v = net(torch.from_numpy(d["x"].astype(np.float32)))
    assert np.abs(p.numpy() - d["policy"]).max() <= 1e-6
    assert np.abs(v.numpy().reshape(-1) - d["value"]).max() <= 1e-6
    assert np.abs(d["value"]).max() < 0.95 and np.median(d["policy"].max(axis=1)) < 0.5


def test_winograd3_algebra_matches_direct_conv(engine_lib):
    """Winograd F(3x3,3x3) as k_wino3h_conv computes it (U from uttt_nn_wino3h_weights, the
    f16 hi + lo halves recombined and unscaled; V = B^T d B on the 5x5 windows of the
    zero-padded board; Y = A^T (U . V) A on 3x3 tiles of 3x3 outputs, nothing cropped) equals
    the direct 3x3 conv."""
    import ctypes
    rng = np.random.RandomState(1)
    w = rng.randn(128, 128, 3, 3).astype(np.float32)
    uh = np.zeros(25 * 128 * 128 * 2, np.uint16)
    su = ctypes.c_float(0.0)
    fp = ctypes.POINTER(ctypes.c_float)
    assert engine_lib.uttt_nn_wino3h_weights(w.ctypes.data_as(fp), ctypes.c_void_p(uh.ctypes.data),
                                             ctypes.byref(su)) == 0
    assert su.value > 0 and np.log2(su.value) == int(np.log2(su.value))
    # stored order U[xi][ci/32][hi|lo][co/16][(ci%32)/8][co%16][ci%8] -> (hi, lo)[xi][ci][co]
    h = uh.view(np.float16).astype(np.float64).reshape(25, 4, 2, 8, 4, 16, 8)
    h = h.transpose(2, 0, 1, 4, 6, 3, 5).reshape(2, 25, 128, 128)
    u = (h[0] + h[1]) / su.value
    assert np.abs(h[1]).max() <= np.abs(h[0]).max() * 2.0 ** -10  # lo is the rounding remainder of hi
    BT = np.array([[2, -1, -2, 1, 0], [0, -2, -1, 1, 0], [0, 2, -3, 1, 0], [0, -1, 0, 1, 0], [0, 2, -1, -2, 1]],
                  np.float64)
    AT = np.array([[1, 1, 1, 1, 0], [0, 1, -1, 2, 0], [0, 1, 1, 4, 1]], np.float64)
    x = rng.randn(9, 9, 128)
    xp = np.zeros((11, 11, 128))
    xp[1:10, 1:10] = x
    y = np.zeros((9, 9, 128))
    U = u.astype(np.float64).reshape(5, 5, 128, 128)
    for ty in range(3):
        for tx in range(3):
            d = xp[3 * ty:3 * ty + 5, 3 * tx:3 * tx + 5]
            V = np.einsum("ui,ijc,vj->uvc", BT, d, BT)
            M = np.einsum("uvc,uvco->uvo", V, U)
            y[3 * ty:3 * ty + 3, 3 * tx:3 * tx + 3] = np.einsum("au,uvo,bv->abo", AT, M, AT)
            # the kernel's fold (round 4): S' = (Z A^T) M along u with Z = [c0 c1 c4]^-1, then
            # S = Z^-1 S' in the epilogue; the same Y
            ZAT = np.array([[1, 0, 2, -1, 0], [0, 1, -1, 2, 0], [0, 0, 2, 2, 1]], np.float64)
            Zinv = np.array([[1, 1, 0], [0, 1, 0], [0, 1, 1]], np.float64)
            assert np.array_equal(Zinv @ ZAT, AT)
            S = np.einsum("za,avo->zvo", Zinv, np.einsum("au,uvo->avo", ZAT, M))
            assert np.allclose(np.einsum("avo,bv->abo", S, AT), y[3 * ty:3 * ty + 3, 3 * tx:3 * tx + 3], rtol=1e-12,
                               atol=1e-9)
    direct = np.zeros((9, 9, 128))
    for ky in range(3):
        for kx in range(3):
            direct += np.einsum("rsc,oc->rso", xp[ky:ky + 9, kx:kx + 9], w[:, :, ky, kx].astype(np.float64))
    assert np.abs(y - direct).max() < 1e-5 * np.abs(direct).max()


def test_main_board_line_check_is_the_reference_eight_compares(uttt_cpp_mod):
    """win9 (uttt_bits.h) is written as shifted ANDs for the rows and columns (round 5); is_lose reads it on the
    opponent's main board (uttt_game.cpp:77-79), so every one of the 512 masks there must give the reference's
    eight-line check (uttt_game.cpp:35-61), and next() must find a small-board win for every cell of every
    board shape (it runs win9 on the board just played, with the small-range divisions by 9 and 27)."""
    m = uttt_cpp_mod
    lines = (0x007, 0x038, 0x1C0, 0x049, 0x092, 0x124, 0x111, 0x054)
    empty = [[0] * 9 for _ in range(9)]
    for mask in range(512):
        main_e = [(mask >> i) & 1 for i in range(9)]
        s = m.State(empty, empty, [0] * 9, main_e, -1)
        assert s.is_lose() == any((mask & x) == x for x in lines), mask
    # the mover completes a line on small board b by playing cell c: the board is won in the next state
    for b in range(9):
        for line in lines:
            for c in range(9):
                if not (line >> c) & 1:
                    continue
                own = [row[:] for row in empty]
                for i in range(9):
                    if (line >> i) & 1 and i != c:
                        own[b][i] = 1
                s = m.State(own, empty, [0] * 9, [0] * 9, b)
                nx = s.next(9 * b + c)
                assert nx.main_board_enemy_pieces[b] == 1, (b, line, c)

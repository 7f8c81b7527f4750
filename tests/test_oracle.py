"""Pins the CPU oracle (oracle/uttt_oracle.c) to the reference's own outputs:
the golden fixtures made by tests/golden/make_golden.py from the reference
C++ (compiled from its sources) and the reference Python driver. When the
reference build is present (build container only), also cross-checks the
oracle against it live on fresh random positions."""
import random

import numpy as np
import pytest

from conftest import golden


def _state(core, d, i, prefix=""):
    return core.OrState.from_arrays(d[prefix + "pieces"][i].reshape(9, 9), d[prefix + "enemy"][i].reshape(9, 9),
                                    d[prefix + "main_p"][i], d[prefix + "main_e"][i], int(d[prefix + "active"][i]))


def test_rules_match_reference(oracle_lib):
    core = oracle_lib
    d = golden("rules.npz")
    n = len(d["n_legal"])
    assert n > 5000
    for i in range(n):
        s = _state(core, d, i)
        legal = s.legal_actions()
        assert len(legal) == d["n_legal"][i]
        assert np.array_equal(np.nonzero(d["legal"][i])[0], legal)
        fl = int(s.is_lose()) | int(s.is_draw()) << 1 | int(s.is_done()) << 2 | int(s.is_first_player()) << 3
        assert fl == d["flags"][i]
        assert np.array_equal(s.tensor_hwc(), d["tensor"][i].astype(np.float32))
        a = int(d["action"][i])
        if a >= 0 and i + 1 < n and d["game"][i + 1] == d["game"][i]:
            nx = s.next(a).arrays()
            assert np.array_equal(nx[0].reshape(81), d["pieces"][i + 1])
            assert np.array_equal(nx[1].reshape(81), d["enemy"][i + 1])
            assert np.array_equal(nx[2], d["main_p"][i + 1]) and np.array_equal(nx[3], d["main_e"][i + 1])
            assert nx[4] == d["active"][i + 1]


def test_unvalidated_next_matches_reference(oracle_lib):
    core = oracle_lib
    d = golden("rules.npz")
    for i in range(len(d["odd_action"])):
        s = _state(core, d, i, "odd_")
        nx = s.next(int(d["odd_action"][i])).arrays()
        assert np.array_equal(nx[0].reshape(81), d["odd_n_pieces"][i])
        assert np.array_equal(nx[1].reshape(81), d["odd_n_enemy"][i])
        assert np.array_equal(nx[2], d["odd_n_main_p"][i]) and np.array_equal(nx[3], d["odd_n_main_e"][i])
        assert nx[4] == d["odd_n_active"][i]


def test_search_matches_reference(oracle_lib):
    core = oracle_lib
    d = golden("search.npz")
    assert int(d["uniq"].max()) == 1  # one unique leaf per flush
    for r in range(len(d["n"])):
        s = _state(core, d, int(d["pos"][r]), "pos_")
        sc, vi, st = core.pv_mcts_scores_hash(s, float(d["temp"][r]), int(d["sims"][r]), int(d["batch"][r]))
        n = int(d["n"][r])
        assert sc.size == n
        assert np.array_equal(sc.view(np.uint32), d["scores"][r][:n].view(np.uint32)), r
        assert st.flushes == d["flushes"][r] and st.evals == d["evals"][r]


def test_selfplay_matches_reference_driver(oracle_lib):
    """self_play_cpp.play (reference Python + reference uttt_cpp) with np.random.seed(seed)."""
    core = oracle_lib
    d = golden("selfplay.npz")
    off = 0
    for g, (seed, ln) in enumerate(zip(d["seeds"], d["lengths"])):
        o = core.self_play_game_hash(int(seed), 1.0, 50, 8)
        assert len(o["actions"]) == ln
        sl = slice(off, off + ln)
        assert np.array_equal(o["tensors"], d["tensors"][sl].astype(np.float32))
        assert np.array_equal(o["policies"].view(np.uint64), d["policies"][sl].view(np.uint64))
        assert np.array_equal(o["actions"], d["actions"][sl].astype(np.int32))
        assert np.array_equal(o["values"], d["values"][sl].astype(np.int32))
        off += ln


def test_numpy_reductions_and_rng(oracle_lib):
    core = oracle_lib
    rng = np.random.RandomState(3)
    for n in list(range(1, 140)) + [300, 1000]:
        a = rng.rand(n) * rng.choice([1e-3, 1.0, 1e3], size=n)
        assert core.np_pairwise_sum(a) == np.sum(a), n
    for seed in (0, 1, 1234, 2**32 - 1):
        m = core.MT(seed)
        ref = np.random.RandomState(seed)
        for _ in range(1500):  # crosses the 624-word twist twice
            assert m.double() == ref.random_sample()
    # choice(p=...) over a few distributions with zeros
    for seed in range(50):
        ref = np.random.RandomState(seed)
        m = core.MT(seed)
        p = rng.rand(rng.randint(1, 82))
        p[rng.rand(p.size) < 0.3] = 0.0
        if p.sum() == 0:
            p[0] = 1.0
        p = p / np.sum(p)
        pol, idx = core.policy_and_sample(m, p.astype(np.float32))
        s = p.astype(np.float32).astype(np.float64)
        s = s / np.sum(s)
        assert np.array_equal(pol, s)
        assert idx == ref.choice(np.arange(p.size), p=s)


def test_to_string_fixture_format(oracle_lib):
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "to_string.json")) as f:
        items = json.load(f)
    assert len(items) > 10 and all("Main Board Status" in it["text"] for it in items)


def test_oracle_vs_compiled_reference_live(oracle_lib):
    """Only where oracle/_ref was built from /root/reference (build container / box snapshot)."""
    from oracle import ref
    if not ref.available():
        pytest.skip("oracle/_ref not built")
    core = oracle_lib
    rng = random.Random(99)
    checked = 0
    for g in range(40):
        s = core.OrState.initial()
        while not s.is_done():
            legal = s.legal_actions()
            if rng.random() < 0.15:
                S, B = rng.choice([(50, 8), (20, 3), (100, 16), (12, 1)])
                tau = rng.choice([1.0, 0.0])
                a, _, _ = core.pv_mcts_scores_hash(s, tau, S, B)
                b, _ = ref.search_hash(s.arrays(), tau, S, B)
                assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
                checked += 1
            s = s.next(rng.choice(legal))
    assert checked > 50


# ---------------------------------------------------------------- arena path --
def _pos_state(core, d, i):
    return core.OrState.from_arrays(d["pos_pieces"][i].reshape(9, 9), d["pos_enemy"][i].reshape(9, 9),
                                    d["pos_main_p"][i], d["pos_main_e"][i], int(d["pos_active"][i]))


def test_oracle_python_mcts_matches_reference_pv_mcts(oracle_lib):
    """or_pv_mcts_scores_py == the reference's pv_mcts.pv_mcts_scores (Python semantics,
    SURVEY App. B) on 42 positions x 7 (S, B) x 3 temperatures, float64 bits; where the
    reference raises ZeroDivisionError (S <= B) the oracle reports no root child visit."""
    core = oracle_lib
    d = golden("pvpy.npz")
    for r in range(len(d["n"])):
        st = _pos_state(core, d, int(d["pos"][r]))
        sc, vis, _ = core.pv_mcts_scores_py_hash(st, float(d["temp"][r]), int(d["sims"][r]), int(d["batch"][r]))
        n = int(d["n"][r])
        if n < 0:
            assert sc is None, r
            continue
        assert sc is not None and sc.size == n, r
        assert np.array_equal(sc.view(np.uint64), d["scores"][r, :n].view(np.uint64)), r


def test_oracle_arena_games_match_reference(oracle_lib):
    """evaluate_network.play with two salted hash players, np.random.seed(seed) per game:
    same moves and same first-player points as the reference."""
    core = oracle_lib
    d = golden("pvpy.npz")
    s0, s1 = (int(x) for x in d["arena_salts"])
    off = 0
    for g in range(len(d["arena_lengths"])):
        first, second = (s0, s1) if g % 2 == 0 else (s1, s0)
        point, acts = core.evaluate_play_hash(int(d["arena_seeds"][g]), first, second)
        n = int(d["arena_lengths"][g])
        assert np.array_equal(acts, d["arena_actions"][off:off + n].astype(np.int32)), g
        assert point == d["arena_points"][g], g
        off += n


def test_oracle_python_self_play_matches_reference(oracle_lib):
    """self_play.py play() (Python PV-MCTS self-play, BASELINE configs[0]) after
    np.random.seed(seed): inputs, float64 policies (bits) and first-player values."""
    core = oracle_lib
    d = golden("pvpy.npz")
    off = 0
    for g in range(len(d["sp_lengths"])):
        n = int(d["sp_lengths"][g])
        r = core.self_play_game_py_hash(int(d["sp_seeds"][g]))
        sl = slice(off, off + n)
        assert len(r["values"]) == n, g
        assert np.array_equal(r["tensors"].astype(np.uint8), d["sp_tensors"][sl]), g
        assert np.array_equal(r["policies"].view(np.uint64), d["sp_policies"][sl].view(np.uint64)), g
        assert np.array_equal(r["values"], d["sp_values"][sl]), g
        off += n

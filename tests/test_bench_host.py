"""CPU tests of bench.py's measurement bookkeeping (no GPU): the tree-kernel rooflines with and without the
fused hash rounds, and the FETCH_SIZE calibration it applies to the PMC traffic."""
import importlib
import os
import sys

from conftest import REPO


def _bench():
    sys.path.insert(0, REPO)
    try:
        return importlib.import_module("bench")
    finally:
        sys.path.remove(REPO)


STATS = {"select": {"ms": 2.6, "launches": 100, "bytes": 100 * 3_000_000},
         "apply": {"ms": 0.05, "launches": 10, "bytes": 90 * 2_000_000}}


def test_fused_rounds_give_one_roofline_with_both_kernels_bytes(monkeypatch):
    b = _bench()
    monkeypatch.delenv("UTTT_FUSED_ROUNDS", raising=False)
    sel, app = b.tree_rooflines(STATS, 4096, "hash", 50, "pmc_select_tree.json", "pmc_apply_tree.json")
    assert sel["kernel"].startswith("k_round")
    assert sel["algo_bytes_per_launch"] == round((100 * 3_000_000 + 90 * 2_000_000) / 110)
    assert sel["event_avg_launch_us"] == round((2.6 + 0.05) * 1e3 / 110, 2)
    assert sel["fused"]["apply_bytes"] == 90 * 2_000_000 and sel["fused"]["k_apply_launches"] == 10
    assert app["fused_into"] == "k_round" and "unit" not in app  # no roofline of its own


def test_unfused_rounds_and_network_rounds_keep_two_kernels(monkeypatch):
    b = _bench()
    monkeypatch.setenv("UTTT_FUSED_ROUNDS", "0")
    sel, app = b.tree_rooflines(STATS, 4096, "hash", 50, None, None)
    assert sel["kernel"].startswith("k_select") and app["kernel"].startswith("k_apply")
    assert sel["algo_bytes_per_launch"] == 3_000_000 and app["algo_bytes_per_launch"] == 18_000_000
    monkeypatch.delenv("UTTT_FUSED_ROUNDS")
    sel, app = b.tree_rooflines(STATS, 2048, "fused", 50, None, None)  # the network rounds are never fused
    assert sel["kernel"].startswith("k_select") and app["kernel"].startswith("k_apply")


def test_fetch_size_correction_is_the_committed_calibration():
    b = _bench()
    ff = b.fetch_factor()
    assert ff is not None and abs(ff["factor"] - 1.8043) < 1e-3
    lo, hi = ff["bounds"]
    assert 0.2 < lo < 0.3 and 1.9 < hi < 2.1
    assert os.path.exists(os.path.join(REPO, "profiles", "r5", "fetch_cal.json"))

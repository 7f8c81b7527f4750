"""The reference-API drop-ins on the GPU, against the reference's own outputs
(tests/golden, generated from /root/reference's modules): pv_mcts_cpp
(pv_mcts_cpp.py:17-167), self_play_cpp.self_play's .history file
(self_play_cpp.py:104-130) on one process and sharded over two torchrun ranks
(SURVEY §8(e)), and a miniature train_cycle.py (train_cycle.py:21-39: self-play ->
train -> evaluate -> evaluate_best_player) composed from the drop-ins."""
import os
import pickle
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, PKG, REPO, golden

pytestmark = pytest.mark.gpu


def _failure_text(r):
    """A child run's failure: its error lines first (a C++ exception's message sits above the stack trace
    that the tails would keep), then the tails."""
    err = [ln for ln in r.stderr.splitlines() if "rror" in ln and "frame #" not in ln][:12]
    return "\n".join(err) + "\n---\n" + r.stdout[-2000:] + r.stderr[-3000:]


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import uttt_amd
    return uttt_amd


def _golden_history():
    d = golden("selfplay.npz")
    return d, int(d["lengths"].sum())


def _check_history(hist, d, n_games):
    """hist: the pickled list [[x (9,9,3) f32, policy (81,) f64, value int], ...] in game order."""
    n = int(d["lengths"][:n_games].sum())
    assert len(hist) == n
    for i, rec in enumerate(hist):
        x, pol, val = rec
        assert isinstance(x, np.ndarray) and x.dtype == np.float32 and x.shape == (9, 9, 3)
        assert isinstance(pol, np.ndarray) and pol.dtype == np.float64 and pol.shape == (81,)
        assert isinstance(val, int)
        assert np.array_equal(x.reshape(243), d["tensors"][i].astype(np.float32)), i
        assert np.array_equal(pol.view(np.uint64), d["policies"][i].view(np.uint64)), i
        assert val == int(d["values"][i]), i


def test_pv_mcts_cpp_dropin_matches_golden(gpu):
    """pv_mcts_scores_cpp / pv_mcts_action_cpp / check_cpp_compatibility with the hash model
    (a torch module with DualNetwork's call signature, called through the reference's glue):
    scores bit-equal to the reference build's on search.npz; the action is numpy's global
    choice over the renormalised scores."""
    import pv_mcts_cpp
    import uttt_cpp
    from oracle.hashnp import make_hash_model
    assert pv_mcts_cpp.check_cpp_compatibility()
    d = golden("search.npz")
    model = make_hash_model()
    rows = np.nonzero((d["sims"] == 50) & (d["batch"] == 8))[0]
    for r in rows[::3]:
        i = int(d["pos"][r])
        st = uttt_cpp.State(d["pos_pieces"][i].reshape(9, 9).tolist(), d["pos_enemy"][i].reshape(9, 9).tolist(),
                            d["pos_main_p"][i].tolist(), d["pos_main_e"][i].tolist(), int(d["pos_active"][i]))
        tau = float(d["temp"][r])
        sc = pv_mcts_cpp.pv_mcts_scores_cpp(model, st, tau, 50, 8)
        n = int(d["n"][r])
        assert sc.shape == (n,)
        assert np.array_equal(sc.astype(np.float32).view(np.uint32), d["scores"][r][:n].view(np.uint32)), r
        if tau == 1.0:
            act = pv_mcts_cpp.pv_mcts_action_cpp(model, tau, 50, 8)
            np.random.seed(77)
            a = act(st)
            legal = st.legal_actions()
            s = sc / np.sum(sc)
            np.random.seed(77)
            assert a == np.random.choice(legal, p=s)


def test_pv_mcts_cpp_fused_path_for_dual_network(gpu):
    """For a DualNetwork the drop-in's callback evaluates the flush's states on the fused HIP
    evaluator (no HWC->NCHW tensor round trip); its outputs are the network's within 1e-5,
    and the search returns a valid distribution over the legal moves."""
    import pv_mcts_cpp
    import torch
    import uttt_cpp
    from uttt_amd.model import calibrated_network
    net = calibrated_network(os.path.join(GOLDEN, "netcal.npz"), "cuda")
    f = pv_mcts_cpp.make_inference_func(net)
    assert f.__name__ == "fused_inference"
    s = uttt_cpp.State()
    states = [s, s.next(40), s.next(40).next(36)]
    out = f(states)
    x = torch.from_numpy(np.stack([np.asarray(t.to_input_tensor(), np.float32).reshape(9, 9, 3)
                                   for t in states]).transpose(0, 3, 1, 2).copy()).cuda()
    with torch.no_grad():
        p, v = net(x)
    for i, (pi, vi) in enumerate(out):
        assert np.abs(pi - p[i].cpu().numpy()).max() <= 1e-5 and abs(vi - float(v[i, 0])) <= 1e-5
    sc = pv_mcts_cpp.pv_mcts_scores_cpp(net, states[1], 1.0, 50, 8)
    assert len(sc) == len(states[1].legal_actions()) and abs(float(np.sum(sc)) - 1.0) < 1e-5


def test_self_play_cpp_writes_reference_history(gpu, tmp_path):
    """self_play_cpp.self_play(): all games concurrently, one .history pickle whose records
    (inputs, float64 policy bits, values, types) equal the reference driver's games
    (selfplay.npz: the reference's self_play_cpp.play after np.random.seed(1234 + g))."""
    import self_play_cpp
    from oracle.hashnp import make_hash_model
    d, _ = _golden_history()
    ng = len(d["lengths"])
    path = self_play_cpp.self_play(n_games=ng, seed_base=int(d["seeds"][0]), model=make_hash_model(),
                                   out_dir=str(tmp_path), slots=7)
    assert os.path.dirname(path) == str(tmp_path) and path.endswith(".history")
    with open(path, "rb") as fh:
        hist = pickle.load(fh)  # written by this test
    _check_history(hist, d, ng)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_self_play_cpp_sharded_over_two_ranks(gpu, tmp_path):
    """torchrun, 2 ranks sharing the GPU (gloo for the gather): each rank plays its block of game
    ids, rank 0 gathers and writes ONE .history equal to the single-process file and the
    reference's games."""
    d, _ = _golden_history()
    ng = len(d["lengths"])
    env = dict(os.environ, UTTT_DIST_BACKEND="gloo", PYTHONPATH=REPO)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "tests", "sharded_selfplay_main.py"), str(tmp_path), str(ng), str(int(d["seeds"][0]))]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, cwd=REPO)
    assert r.returncode == 0, _failure_text(r)
    files = sorted(p for p in os.listdir(tmp_path) if p.endswith(".history"))
    assert len(files) == 1, files
    with open(os.path.join(tmp_path, files[0]), "rb") as fh:
        hist = pickle.load(fh)  # written by this test's child
    _check_history(hist, d, ng)


def test_rccl_one_rank_data_path_and_ddp(gpu):
    """The RCCL ("nccl") branches on the device, one torchrun rank (two RCCL ranks cannot share one
    GPU; more ranks are rehearsed with gloo above): self_play_sharded's gather_records (all_gather of
    device tensors) returns the single-process games bit for bit, broadcast_int round-trips, and DDP
    steps whose gradient all-reduce runs over RCCL train (tests/rccl_one_rank_main.py)."""
    env = dict(os.environ, PYTHONPATH=REPO)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "tests", "rccl_one_rank_main.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, cwd=REPO)
    assert r.returncode == 0, _failure_text(r)
    assert "RCCL-OK" in r.stdout


def test_flat_dp_train_network_two_ranks(gpu, tmp_path):
    """train_network under torchrun on the GPU (the opt-in data-parallel form, UTTT_TRAIN_DP=flat: the
    per-rank step as two captured graphs around one flat gradient all-reduce), 2 ranks sharing the GPU over
    gloo, different start weights per rank (rank 0's are broadcast): identical weights, averaged BatchNorm
    running statistics and losses on both ranks (tests/dp_flat_two_ranks_main.py)."""
    import torch
    env = dict(os.environ, PYTHONPATH=REPO)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "tests", "dp_flat_two_ranks_main.py"), str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, cwd=REPO)
    assert r.returncode == 0, _failure_text(r)
    m0 = torch.load(tmp_path / "m0.pt", weights_only=True)
    m1 = torch.load(tmp_path / "m1.pt", weights_only=True)
    for k in m0["sd"]:
        assert torch.equal(m0["sd"][k], m1["sd"][k]), k
    assert m0["losses"] == m1["losses"] and all(np.isfinite(m0["losses"]))


def test_bench_multi_rank_path(gpu):
    """bench.py's N>1 path (what the driver's scaling run executes) rehearsed with 2 torchrun ranks
    on the one GPU (gloo instead of RCCL): per-rank game blocks, barrier + max-over-ranks timing,
    the whole-job value and one JSON line from rank 0."""
    import json
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--age", "3", "--games", "256",
           "--rehearse-shared-gpu", "--no-variants", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, _failure_text(r)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and "rehearsal" in out["config"]
    # 2 ranks x 256 games x 50 sims per step, whole-job over the slowest rank's time
    assert out["value"] > 0 and abs(out["value"] * out["ms_per_step"] / 1e3 - 2 * 256 * 50) < 1e-3 * 2 * 256 * 50
    # the value's steps run with no events in them; the kernel statistics come from a separate pass
    ip = out["instrumented_pass"]
    assert ip["steps"] == 2 and ip["value"] > 0 and out["roofline"]["launches"] > 0


def test_mini_train_cycle(gpu, tmp_path, monkeypatch):
    """train_cycle.py:21-39 in miniature, every step through this build's drop-ins in a fresh
    working directory: dual_network() -> self_play() (fused evaluator, .history) ->
    train_network() (1 epoch) -> evaluate_network() (2 arena games) -> evaluate_best_player()
    (2 games VS_Random)."""
    import dual_network
    import evaluate_best_player
    import evaluate_network
    import self_play_cpp
    import train_network
    from uttt_amd import train as _train
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(self_play_cpp, "SP_GAME_COUNT", 8)
    monkeypatch.setattr(train_network, "RN_EPOCHS", 1)
    monkeypatch.setattr(evaluate_network, "EN_GAME_COUNT", 2)
    monkeypatch.setattr(evaluate_best_player, "EP_GAME_COUNT", 2)
    dual_network.dual_network()
    assert os.path.exists("model/best.pth")
    path = self_play_cpp.self_play()
    with open(path, "rb") as fh:
        hist = pickle.load(fh)  # written by this test
    assert len(hist) >= 8 * 9 and all(r[0].shape == (9, 9, 3) for r in hist)
    train_network.train_network()
    assert os.path.exists("model/latest.pth")
    promoted = evaluate_network.evaluate_network()
    assert promoted in (True, False)
    pt = evaluate_best_player.evaluate_best_player()
    assert 0.0 <= pt <= 1.0
    assert _train.RN_EPOCHS == 100  # the module constant itself is untouched

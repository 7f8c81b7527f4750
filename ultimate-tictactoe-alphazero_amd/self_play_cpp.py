"""Drop-in for the reference's self_play_cpp.py, on the MI355X engine.

Same names and constants (self_play_cpp.py:26-31), same .history schema
(:59, :95-99, :125-130). Differences, by design:

* ``self_play()`` plays all SP_GAME_COUNT games concurrently (the reference
  plays them one after another). Game g draws its moves from
  ``np.random.RandomState(seed_base + g)``'s stream — equal to the reference's
  ``play()`` after ``np.random.seed(seed_base + g)``. seed_base defaults to a
  draw from numpy's global RNG (the reference is unseeded).
* Under ``torchrun --nproc-per-node N`` (WORLD_SIZE > 1) every rank plays a
  contiguous block of game ids on its own GPU, the compact records are
  gathered to rank 0 over RCCL, and rank 0 writes ONE .history file (the
  reference's train_network.py reads only the newest file). The file is the
  same for any N (game g depends only on g).
* ``play(model)`` runs one game on the engine and draws from (and advances)
  numpy's global RNG exactly as the reference does.
* For a DualNetwork the leaf evaluator is the fused HIP kernels (nnfast;
  value/policy within 1e-5 of the model's own forward); any other model is
  called as model(x). UTTT_EVALUATOR=torch forces the model call.
"""
import os
import pickle
import sys
import time
from datetime import datetime

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
try:
    import uttt_cpp  # noqa: F401
    CPP_AVAILABLE = True
    print("Using C++ backend for MCTS")
except ImportError:
    CPP_AVAILABLE = False
    print("C++ backend not available")

from uttt_amd.model import DualNetwork  # noqa: E402
from uttt_amd.distributed import broadcast_int, init_from_env, self_play_sharded  # noqa: E402
from uttt_amd.history import write_history_file  # noqa: E402
from uttt_amd.selfplay import SelfPlay, default_lanes, history_from_records  # noqa: E402

SP_GAME_COUNT = 500
SP_TEMPERATURE = 1.0
PV_EVALUATE_COUNT = 50
MCTS_BATCH_SIZE = 8

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
_single = {}
# wall-clock seconds of the last self_play() call's phases (tools/bench_cycle.py)
LAST_TIMINGS = {}


def _fingerprint(model):
    return tuple((t.data_ptr(), t._version) for t in model.state_dict().values())


def _runner(model, slots):
    """One cached single-game runner per model (rebuilt when its weights change)."""
    key = (id(model), slots, _fingerprint(model))
    r = _single.get("runner") if _single.get("key") == key else None
    if r is None:
        _single.clear()
        r = SelfPlay(slots, PV_EVALUATE_COUNT, MCTS_BATCH_SIZE, SP_TEMPERATURE, model=model)
        _single.update(key=key, runner=r)
    return r


def play(model, use_cpp=True):
    """One self-play game (self_play_cpp.py:34-101) on numpy's global RNG."""
    if not (use_cpp and CPP_AVAILABLE):
        raise RuntimeError("the engine backend is required (build ultimate-tictactoe-alphazero_amd)")
    model = model.to(device).eval()
    r = _runner(model, 1)
    r.begin(0, 1, 0)
    st = np.random.get_state()
    r.engine.set_rng(st[1], st[2], slot=0)
    while r.step():
        pass
    key, pos = r.engine.get_rng(0)
    np.random.set_state((st[0], key, pos, st[3], st[4]))
    return history_from_records(r.records())


def _history_path(out_dir):
    now = datetime.now()
    os.makedirs(out_dir, exist_ok=True)
    return os.path.join(out_dir, "{:04}{:02}{:02}{:02}{:02}{:02}.history".format(
        now.year, now.month, now.day, now.hour, now.minute, now.second))


def write_history(history, out_dir="./data"):
    """A history list -> ./data/YYYYmmddHHMMSS.history (self_play_cpp.py:125-130)."""
    path = _history_path(out_dir)
    with open(path, mode="wb") as f:
        pickle.dump(history, f)
    return path


def write_history_records(records, out_dir="./data"):
    """The same file from game records, written by uttt_amd.history (loads to the list write_history
    would store, without pickling ply by ply)."""
    path = _history_path(out_dir)
    write_history_file(records, path)
    return path


def self_play(use_cpp=True, n_games=None, slots=None, seed_base=None, model_path="./model/best.pth",
              out_dir="./data", model=None, lanes=None):
    """SP_GAME_COUNT games -> ./data/YYYYmmddHHMMSS.history (self_play_cpp.py:104-130). Returns the
    file's path (on rank 0 under torchrun; None on the other ranks)."""
    if not (use_cpp and CPP_AVAILABLE):
        raise RuntimeError("the engine backend is required (build ultimate-tictactoe-alphazero_amd)")
    rank, world, local = init_from_env()
    dev = torch.device("cuda", local) if torch.cuda.is_available() else device
    n_games = SP_GAME_COUNT if n_games is None else n_games
    if model is None:
        model = DualNetwork().to(dev)
        model.load_state_dict(torch.load(model_path, map_location=dev, weights_only=True))
    model = model.to(dev).eval()
    if world > 1:
        seed_base = broadcast_int(int(np.random.randint(0, 2**31 - 1)) if seed_base is None else seed_base)
    elif seed_base is None:
        seed_base = int(np.random.randint(0, 2**31 - 1))
    slots = min(n_games, 4096) if slots is None else slots

    def progress(done, total):
        if rank == 0:
            print(f"\rSelfPlay {done}/{total} (Backend: HIP, {world} GPU)", end="")

    LAST_TIMINGS.clear()
    t0 = time.perf_counter()
    if world > 1:
        recs = self_play_sharded(model, n_games, slots, seed_base, PV_EVALUATE_COUNT, MCTS_BATCH_SIZE,
                                 SP_TEMPERATURE, lanes=lanes, progress=progress, timings=LAST_TIMINGS)
    else:
        n_lanes = default_lanes(slots) if lanes is None else lanes
        r = SelfPlay(slots, PV_EVALUATE_COUNT, MCTS_BATCH_SIZE, SP_TEMPERATURE, device=dev.index, model=model,
                     lanes=n_lanes)
        LAST_TIMINGS["setup_s"] = time.perf_counter() - t0
        LAST_TIMINGS["games_s"] = r.run(0, n_games, seed_base, progress)
        LAST_TIMINGS["sims"] = r.sims
        t1 = time.perf_counter()
        recs = r.records()
        LAST_TIMINGS["records_s"] = time.perf_counter() - t1
    path = None
    if rank == 0:
        print("")
        t1 = time.perf_counter()
        path = write_history_records(recs, out_dir)
        LAST_TIMINGS.update(history_write_s=time.perf_counter() - t1, plies=sum(len(r["actions"]) for r in recs),
                            history_bytes=os.path.getsize(path))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    LAST_TIMINGS["total_s"] = time.perf_counter() - t0
    return path


if __name__ == "__main__":
    self_play()

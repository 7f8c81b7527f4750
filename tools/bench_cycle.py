#!/usr/bin/env python3
"""BASELINE configs[4] on this build: one full train_cycle.py iteration (train_cycle.py:21-39) through
the drop-ins with the reference's constants, in a fresh working directory, every phase timed:

  dual_network()          ./model/best.pth (seed-0 init)                 dual_network.py:125-135
  self_play()             SP_GAME_COUNT = 500 games -> ./data/*.history  self_play_cpp.py:104-130
  train_network()         RN_EPOCHS = 100, batch 128, Adam               train_network.py:41-125
  evaluate_network()      EN_GAME_COUNT = 50 arena games                 evaluate_network.py:62-104
  evaluate_best_player()  EP_GAME_COUNT = 10 games VS_Random             evaluate_best_player.py:20-98

The reference publishes (README.md:289-299, RTX 4070 Ti + Ryzen 7 5800X): self-play of 500 games 2 min,
one training epoch 2 s, a full learning cycle 4 min. One JSON line (also written to --out).
usage: python tools/bench_cycle.py [--workdir DIR] [--out profiles/r3/cycle.json] [--games 500] [--epochs 100]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")
sys.path[:0] = [REPO, PKG]


def main():
    ap = argparse.ArgumentParser()
    import tempfile
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "uttt_cycle_wd"),
                    help="scratch working directory (./model, ./data); outside gpurun_out (64 MiB cap)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--games", type=int, default=None, help="SP_GAME_COUNT override (default: the reference's 500)")
    ap.add_argument("--epochs", type=int, default=None, help="RN_EPOCHS override (default: the reference's 100)")
    ap.add_argument("--arena-games", type=int, default=None, help="EN_GAME_COUNT override (default 50)")
    args = ap.parse_args()
    import shutil

    import numpy as np
    import torch
    os.makedirs(args.workdir, exist_ok=True)
    for sub in ("model", "data"):
        shutil.rmtree(os.path.join(args.workdir, sub), ignore_errors=True)
    os.chdir(args.workdir)
    t_import = time.perf_counter()
    import dual_network
    import evaluate_best_player
    import evaluate_network
    import self_play_cpp
    import train_network
    if args.games:
        self_play_cpp.SP_GAME_COUNT = args.games
    if args.epochs:
        train_network.RN_EPOCHS = args.epochs
    if args.arena_games:
        evaluate_network.EN_GAME_COUNT = args.arena_games
    out = {"metric": "train_cycle.py iteration wall time (s), BASELINE configs[4] on 1 GPU",
           "config": {"SP_GAME_COUNT": self_play_cpp.SP_GAME_COUNT, "PV_EVALUATE_COUNT": self_play_cpp.PV_EVALUATE_COUNT,
                      "MCTS_BATCH_SIZE": self_play_cpp.MCTS_BATCH_SIZE, "RN_EPOCHS": train_network.RN_EPOCHS,
                      "BATCH_SIZE": train_network.BATCH_SIZE, "EN_GAME_COUNT": evaluate_network.EN_GAME_COUNT,
                      "EP_GAME_COUNT": evaluate_best_player.EP_GAME_COUNT},
           "n_gpus": 1, "device": torch.cuda.get_device_name(0), "phases": {},
           "train_precision": os.environ.get("UTTT_TRAIN_PRECISION", "fp32")}
    out["import_s"] = round(time.perf_counter() - t_import, 3)
    torch.manual_seed(0)
    np.random.seed(0)
    ph = out["phases"]

    def timed(name, fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ph[name] = {"s": round(time.perf_counter() - t, 3)}
        print(f"[cycle] {name}: {ph[name]['s']} s", file=sys.stderr, flush=True)
        return r

    t0 = time.perf_counter()
    timed("dual_network", dual_network.dual_network)
    timed("self_play", self_play_cpp.self_play)
    ph["self_play"].update({k: (round(v, 3) if isinstance(v, float) else v)
                            for k, v in self_play_cpp.LAST_TIMINGS.items()})
    sp = self_play_cpp.LAST_TIMINGS
    if sp.get("games_s"):
        ph["self_play"]["sims_per_s"] = round(sp["sims"] / sp["games_s"], 1)
    timed("train_network", train_network.train_network)
    tt = train_network.LAST_TIMINGS
    ph["train_network"].update({k: (round(v, 4) if isinstance(v, float) else v) for k, v in tt.items()})
    ph["train_network"]["s_per_epoch"] = round(tt["train_s"] / tt["epochs"], 3)
    ph["train_network"]["samples_per_s"] = round(tt["samples"] * tt["epochs"] / tt["train_s"], 1)
    promoted = timed("evaluate_network", evaluate_network.evaluate_network)
    ph["evaluate_network"]["promoted"] = bool(promoted)
    timed("evaluate_best_player", evaluate_best_player.evaluate_best_player)
    ph["evaluate_best_player"]["runs_in_reference_cycle"] = bool(promoted)
    total = time.perf_counter() - t0
    out["cycle_s"] = round(total, 3)
    out["cycle_s_reference_order"] = round(total - (0 if promoted else ph["evaluate_best_player"]["s"]), 3)
    out["reference_published"] = {"self_play_500_games_s": 120, "train_epoch_s": 2.0, "cycle_s": 240,
                                  "source": "README.md:289-299 (RTX 4070 Ti + Ryzen 7 5800X)"}
    out["vs_reference"] = {"self_play": round(120 / ph["self_play"]["s"], 2),
                           "train_epoch": round(2.0 / ph["train_network"]["s_per_epoch"], 2),
                           "cycle": round(240 / out["cycle_s_reference_order"], 2),
                           "note": "reference time / this build's time (higher is faster)"}
    line = json.dumps(out)
    print(line)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(os.path.join(REPO, args.out))), exist_ok=True)
        with open(os.path.join(REPO, args.out), "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()

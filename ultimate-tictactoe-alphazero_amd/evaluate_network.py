"""Drop-in for the reference's evaluate_network.py: latest vs best, EN_GAME_COUNT
games, model0 (latest) moving first in the even games (evaluate_network.py:58-104).

The games run concurrently on the MI355X engine (uttt_amd.arena); game g draws
its moves from RandomState(seed_base + g) with seed_base taken from numpy's
global RNG, where the reference draws every game's moves from the global RNG in
sequence — per-game streams are what lets the games advance together, and with
np.random.seed(seed_base + g) before each reference play() the records match
(tests/test_engine_gpu.py, tests/golden/pvpy.npz). play() keeps the reference's
sequential form for callers that pass their own next_actions.
"""
import os
import sys
from shutil import copy

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import uttt_cpp  # noqa: E402
from uttt_amd import arena  # noqa: E402
from uttt_amd.model import DualNetwork  # noqa: E402

CPP_GAME_AVAILABLE = True
EN_GAME_COUNT = 50
EN_TEMPERATURE = 1.0

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
first_player_point = arena.first_player_point


def play(next_actions):
    state = uttt_cpp.State()
    while True:
        if state.is_done():
            break
        next_action = next_actions[0] if state.is_first_player() else next_actions[1]
        action = next_action(state)
        state = state.next(action)
    return first_player_point(state)


def update_best_player():
    copy("./model/latest.pth", "./model/best.pth")
    print("Change BestPlayer")


def evaluate_network():
    model0 = DualNetwork().to(device)
    model0.load_state_dict(torch.load("./model/latest.pth", map_location=device, weights_only=True))
    model0.eval()
    model1 = DualNetwork().to(device)
    model1.load_state_dict(torch.load("./model/best.pth", map_location=device, weights_only=True))
    model1.eval()
    seed_base = int(np.random.randint(0, 2**31 - EN_GAME_COUNT))

    def progress(done, total):
        print("\rEvaluate {}/{}".format(done, total), end="")

    average_point, _, _ = arena.evaluate_network(model0, model1, EN_GAME_COUNT, EN_TEMPERATURE, seed_base,
                                                 progress=progress)
    print("")
    print("AveragePoint", average_point)
    del model0
    del model1
    if average_point > 0.5:
        update_best_player()
        return True
    return False


if __name__ == "__main__":
    evaluate_network()

"""Drop-in for the reference's self_play.py (the Python self-play: pv_mcts.py
searches, BASELINE.json configs[0]) on the MI355X engine.

  first_player_value(ended_state)  self_play.py:20-25
  write_data(history)              self_play.py:28-35
  play(model)                      self_play.py:66-99 (one game, numpy's global RNG)
  self_play()                      self_play.py:102-127 (SP_GAME_COUNT games)

self_play() runs all games concurrently (uttt_amd.arena.self_play_py): game g
draws from RandomState(seed_base + g), seed_base taken from numpy's global RNG;
play() keeps the reference's sequential, global-RNG form. Records match the
reference's play() after np.random.seed(seed) (tests/golden/pvpy.npz).
"""
import os
import pickle
import sys
from datetime import datetime

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import uttt_cpp  # noqa: E402
from pv_mcts import pv_mcts_scores  # noqa: E402
from uttt_amd import arena  # noqa: E402
from uttt_amd.model import DN_INPUT_SHAPE, DualNetwork  # noqa: E402,F401

DN_OUTPUT_SIZE = 81
SP_GAME_COUNT = 500
SP_TEMPERATURE = 1.0

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
first_player_value = arena.first_player_value


def write_data(history):
    now = datetime.now()
    os.makedirs("./data/", exist_ok=True)
    path = "./data/{:04}{:02}{:02}{:02}{:02}{:02}.history".format(now.year, now.month, now.day, now.hour,
                                                                  now.minute, now.second)
    with open(path, mode="wb") as f:
        pickle.dump(history, f)


def play(model):
    history = []
    state = uttt_cpp.State()
    while True:
        if state.is_done():
            break
        scores = pv_mcts_scores(model, state, SP_TEMPERATURE)
        policies = [0] * DN_OUTPUT_SIZE
        for action, policy in zip(state.legal_actions(), scores):
            policies[action] = policy
        history.append([np.asarray(state.to_input_tensor(), np.float64).reshape(9, 9, 3), policies, None])
        action = np.random.choice(state.legal_actions(), p=scores)
        state = state.next(action)
    value = first_player_value(state)
    for i in range(len(history)):
        history[i][2] = value
        value = -value
    return history


def self_play():
    model = DualNetwork().to(device)
    model.load_state_dict(torch.load("./model/best.pth", map_location=device, weights_only=True))
    model.eval()
    seed_base = int(np.random.randint(0, 2**31 - SP_GAME_COUNT))

    def progress(done, total):
        print("\rSelfPlay {}/{}".format(done, total), end="")

    games = arena.self_play_py(model, SP_GAME_COUNT, seed_base, SP_TEMPERATURE, progress=progress)
    print("")
    history = [rec for g in games for rec in g]
    write_data(history)
    del model


if __name__ == "__main__":
    self_play()

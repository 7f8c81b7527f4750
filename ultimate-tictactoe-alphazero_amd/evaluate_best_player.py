"""Drop-in for the reference's evaluate_best_player.py (evaluate_best_player.py:20-98): the best
model's PV-MCTS player (pv_mcts.pv_mcts_action at temperature 0, on the MI355X engine with the
Python-search semantics and the fused HIP evaluator) against the random player, EP_GAME_COUNT
games alternating the first move, printing "VS_Random <average point>" for the training monitors.
The alpha-beta and plain-MCTS opponents are disabled in the reference too (:86-93)."""
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import uttt_cpp  # noqa: E402
from pv_mcts import pv_mcts_action  # noqa: E402
from uttt_amd import arena  # noqa: E402
from uttt_amd.model import DualNetwork  # noqa: E402

CPP_GAME_AVAILABLE = True
EP_GAME_COUNT = 10

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
first_player_point = arena.first_player_point


def random_action(state):
    """game.py:234-236 (Python's global `random`)."""
    legal_actions = state.legal_actions()
    return legal_actions[random.randint(0, len(legal_actions) - 1)]


def play(next_actions):
    state = uttt_cpp.State()
    while not state.is_done():
        next_action = next_actions[0] if state.is_first_player() else next_actions[1]
        state = state.next(next_action(state))
    return first_player_point(state)


def evaluate_algorithm_of(label, next_actions):
    total_point = 0
    for i in range(EP_GAME_COUNT):
        if i % 2 == 0:
            total_point += play(next_actions)
        else:
            total_point += 1 - play(list(reversed(next_actions)))
        print("\rEvaluate {}/{}".format(i + 1, EP_GAME_COUNT), end="")
    print("")
    average_point = total_point / EP_GAME_COUNT
    print(label, average_point)
    return average_point


def evaluate_best_player():
    model = DualNetwork().to(device)
    model.load_state_dict(torch.load("./model/best.pth", map_location=device, weights_only=True))
    model.eval()
    next_pv_mcts_action = pv_mcts_action(model, 0.0)
    point = evaluate_algorithm_of("VS_Random", (next_pv_mcts_action, random_action))
    del model
    return point


if __name__ == "__main__":
    evaluate_best_player()

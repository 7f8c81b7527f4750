"""Drop-in for the reference's pv_mcts.py (the Python PV-MCTS used by
evaluate_network.py / evaluate_best_player.py), backed by the MI355X engine
with UTTT_SEMANTICS_PY:

  predict_batch(model, states_batch)         pv_mcts.py:21-61
  nodes_to_scores(nodes)                     pv_mcts.py:64-68
  pv_mcts_scores(model, state, temperature)  pv_mcts.py:71-181 (one tree, module constants below)
  pv_mcts_action(model, temperature=0)       pv_mcts.py:184-188 (numpy's global RNG)
  boltzman(xs, temperature)                  pv_mcts.py:190-192

Same results as the reference on the same inputs (scores bit for bit; PUCT as
NumPy 2 evaluates the reference's expression), including its
ZeroDivisionError when no root child was visited (S <= B).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import uttt_cpp  # noqa: E402,F401  (in-tree; imports torch first so one HIP runtime serves both)
from uttt_amd.arena import PvMcts, model_evaluator, scores_from_visits  # noqa: E402

PV_EVALUATE_COUNT = 50
MCTS_BATCH_SIZE = 8

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
_SEARCH = {}


def predict_batch(model, states_batch):
    """[(legal priors: float32 normalised by np.sum, or float64 uniform), value]."""
    from uttt_amd.arena import _engine_state
    x = np.stack([np.asarray(_engine_state(s).to_input_tensor(), np.float32).reshape(9, 9, 3) for s in states_batch],
                 axis=0).transpose(0, 3, 1, 2)
    dev = next((p.device for p in model.parameters()), device)
    model.eval()
    with torch.no_grad():
        policies, values = model(torch.FloatTensor(x).to(dev))
    policies = policies.cpu().numpy()
    values = values.cpu().numpy()
    results = []
    for i, state in enumerate(states_batch):
        legal = state.legal_actions()
        lp = policies[i][legal] if legal else []
        total = np.sum(lp)
        if total > 0:
            lp /= total
        elif legal:
            lp = np.ones_like(legal, dtype=float) / len(legal)
        else:
            lp = []
        results.append((lp, values[i][0]))
    return results


def nodes_to_scores(nodes):
    return [c.n for c in nodes]


def _search(evaluate_count):
    key = torch.cuda.current_device()
    s = _SEARCH.get(key)
    if s is None or s.engine.max_sims < evaluate_count:
        s = _SEARCH[key] = PvMcts(1, max(50, evaluate_count))
    return s


def pv_mcts_scores(model, state, temperature):
    s = _search(PV_EVALUATE_COUNT)
    (v,) = s.visits([state], model_evaluator(model, 1, s.engine), PV_EVALUATE_COUNT, MCTS_BATCH_SIZE)
    return scores_from_visits(v, temperature)


def pv_mcts_action(model, temperature=0):
    def pv_mcts_action(state):
        scores = pv_mcts_scores(model, state, temperature)
        return np.random.choice(state.legal_actions(), p=scores)

    return pv_mcts_action


def boltzman(xs, temperature):
    xs = [x ** (1 / temperature) for x in xs]
    return [x / sum(xs) for x in xs]

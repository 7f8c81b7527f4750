"""Drop-in for the reference's pv_mcts_cpp.py (same functions, arguments and
errors), backed by this build's `uttt_cpp` — whose pv_mcts_scores runs the
search on the MI355X engine and calls back here once per flush.

  pv_mcts_scores_cpp(model, state, temperature, evaluate_count=50, batch_size=8)  (pv_mcts_cpp.py:17-89)
  pv_mcts_action_cpp(model, temperature=0, evaluate_count=50, batch_size=8)      (pv_mcts_cpp.py:92-137)
  check_cpp_compatibility()                                                       (pv_mcts_cpp.py:140-167)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
try:
    import uttt_cpp
    CPP_AVAILABLE = True
except ImportError:
    CPP_AVAILABLE = False
    print("Warning: uttt_cpp module not found. Using Python implementation.")

from uttt_amd.model import DN_INPUT_SHAPE  # noqa: E402,F401  (re-exported like the reference)

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _model_device(model):
    for p in model.parameters():
        return p.device
    return device


def make_inference_func(model, evaluator=None):
    """The flush callback: list of uttt_cpp.State -> [(policy (81,) f32, value float)].

    For a DualNetwork (the reference's or this package's) the states go straight to the fused
    HIP evaluator (stem from the packed bitboards, Winograd tower, heads; within 1e-5 of the
    model's own forward, tests/test_engine_gpu.py); for any other model, or with
    evaluator="torch" / UTTT_EVALUATOR=torch, the states' HWC tensors are stacked and moved to
    NCHW as the reference builds them (pv_mcts_cpp.py:47-60) and the model is called."""
    from uttt_amd.nnfast import FusedNetworkEvaluator, evaluator_kind
    if torch.cuda.is_available() and evaluator_kind(model, evaluator) == "fused":
        from uttt_amd import as_states
        dev = _model_device(model)
        dev = dev if dev.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
        box = {}

        def fused_inference(states_list):
            n = len(states_list)
            fe = box.get("fe")
            if fe is None or fe.max_batch < n:
                fe = box["fe"] = FusedNetworkEvaluator(model, None, max_batch=max(64, n), device=dev)
            p, v = fe.forward_states(as_states(states_list))
            p, v = p.cpu().numpy(), v.cpu().numpy()
            return [(p[i], float(v[i])) for i in range(n)]

        fused_inference.fused = True
        return fused_inference
    dev = _model_device(model)

    def inference_func(states_list):
        hwc = np.asarray([s.to_input_tensor() for s in states_list], dtype=np.float32).reshape(-1, 9, 9, 3)
        x = torch.from_numpy(np.ascontiguousarray(hwc.transpose(0, 3, 1, 2))).to(dev)
        with torch.no_grad():
            policies, values = model(x)
        policies = policies.float().cpu().numpy()
        values = values.float().cpu().numpy().reshape(len(states_list), -1)
        return [(policies[i], float(values[i][0])) for i in range(len(states_list))]

    return inference_func


def pv_mcts_scores_cpp(model, state, temperature, evaluate_count=50, batch_size=8):
    if not CPP_AVAILABLE:
        raise RuntimeError("C++ module is not available. Please build uttt_cpp first.")
    model.eval()
    fn = make_inference_func(model)
    # the fused HIP evaluator takes the flush's one distinct state (the k queued copies are identical, no
    # virtual loss); the PyTorch forward gets the reference's k copies (MIOpen's batch-1 convolutions ran
    # slower than its batch-k ones: 13.2 against 11.0 ms of model time per search, profiles/r5/latency_single.json)
    scores = uttt_cpp.pv_mcts_scores(model=fn, state=_to_engine_state(state), temperature=temperature,
                                     evaluate_count=evaluate_count, batch_size=batch_size,
                                     dedup=getattr(fn, "fused", False))
    return np.array(scores)


def _to_engine_state(state):
    if isinstance(state, uttt_cpp.State):
        return state
    return uttt_cpp.State(state.pieces, state.enemy_pieces, state.main_board_pieces, state.main_board_enemy_pieces,
                          state.active_board)


def pv_mcts_action_cpp(model, temperature=0, evaluate_count=50, batch_size=8):
    def action_func(state):
        s = _to_engine_state(state)
        scores = pv_mcts_scores_cpp(model, s, temperature, evaluate_count, batch_size)
        legal = s.legal_actions()
        if len(scores) != len(legal):
            raise ValueError(f"Score size mismatch: scores={len(scores)}, legal_actions={len(legal)}")
        total = np.sum(scores)
        scores = np.ones(len(scores)) / len(scores) if total == 0 else scores / total
        return np.random.choice(legal, p=scores)

    return action_func


def check_cpp_compatibility():
    if not CPP_AVAILABLE:
        print("XX C++ module is NOT available")
        print("   Please run: make -C ultimate-tictactoe-alphazero_amd")
        return False
    print("✅ C++ module is available")
    try:
        s = uttt_cpp.State()
        legal = s.legal_actions()
        print(f"✅ Game logic working (legal actions: {len(legal)})")
        if legal:
            s.next(legal[0])
            print("✅ State transition working")
        print(f"✅ Tensor conversion working (shape: {len(s.to_input_tensor())})")
        return True
    except Exception as e:  # mirror of the reference's reporting
        print(f"XX C++ module test failed: {e}")
        return False


if __name__ == "__main__":
    check_cpp_compatibility()
